"""BASELINE config 4 on one GPU: PATTERN graph-batch data-parallel training with 2, 3 and 4
ranks (3 ranks: uneven 3/3/2-graph shards), each a FRESH child process (never a re-exec of this
GPU-initialised process), gloo standing in for RCCL since the ranks share cuda:0. The overlapped,
count-weighted gradient all-reduce must give every rank the gradient of one process training on
the union batch (`models/pattern_gat.py:18-25`), within 2e-4 of the gradient's
scale — also with an edge-mean attention-norm term weighted by E' counts. RCCL itself runs at
world size 1 (the one GPU) through the same reducer and count_weights with their collectives
forced on. bench.py --gpus 2 must start its two ranks itself."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(world, tmp_path, backend="gloo", loss="bce"):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_pattern_worker.py"),
                                       str(tmp_path), backend, loss], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)


@pytest.mark.parametrize("world,backend,loss", [(2, "gloo", "bce"), (3, "gloo", "bce"),
                                                (4, "gloo", "bce"), (3, "gloo", "bce+norm"),
                                                (1, "nccl", "bce+norm")])
def test_pattern_sharded_gradients_equal_union_batch(world, backend, loss, device, tmp_path):
    sys.path.insert(0, HERE)
    import dist_pattern_worker as W
    from gatx import GATModel
    from gatx.config import data_config
    from gatx.distributed import collate_graphs

    _run_ranks(world, tmp_path, backend, loss)
    # single process, union batch (all graphs in order)
    torch.manual_seed(0)
    model = GATModel(**data_config["PATTERN"]).to(device).train()
    x, ei, y, _ = collate_graphs(W.pattern_graphs(device))
    W.pattern_step_grads(model, x, ei, y, loss=loss)
    ref = {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()}
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npz")
        assert set(got.files) == set(ref)
        for n, g in ref.items():
            err = np.abs(got[n] - g).max()
            assert err <= 2e-4 * max(1.0, np.abs(g).max()), (r, n, err, np.abs(g).max())


def test_bench_gpus2_launches_two_ranks():
    """`python bench.py --gpus 2` (the driver's command form, no launcher around it) starts two
    rank processes itself and reports n_gpus 2 (gloo / one device: the one-GPU stand-in)."""
    import json
    root = os.path.dirname(HERE)
    env = dict(os.environ, GATX_BENCH_BACKEND="gloo", GATX_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps",
                        "3", "--warmup", "1", "--workload", "pattern", "--graphs", "8",
                        "--mode", "train"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=200)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout.decode()[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["value"] > 0
    assert r["config"]["parallelism"] == "graph-batch dp2"
