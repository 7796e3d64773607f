"""BASELINE config 4 on one GPU: PATTERN graph-batch data-parallel training with two ranks, each
a FRESH child process (never a re-exec of this GPU-initialised process), gloo standing in for
RCCL since both ranks share cuda:0. The overlapped, count-weighted gradient all-reduce must give
every rank the gradient of one process training on the union batch (`models/pattern_gat.py:18-25`,
SURVEY.md §8e), within 2e-4 of the gradient's scale."""
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


@pytest.mark.parametrize("world", [2])
def test_pattern_sharded_gradients_equal_union_batch(world, device, tmp_path):
    sys.path.insert(0, HERE)
    import dist_pattern_worker as W
    from gatx import GATModel
    from gatx.config import data_config
    from gatx.distributed import collate_graphs

    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_pattern_worker.py"),
                                       str(tmp_path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)

    # single process, union batch (all graphs in order)
    torch.manual_seed(0)
    model = GATModel(**data_config["PATTERN"]).to(device).train()
    x, ei, y, _ = collate_graphs(W.pattern_graphs(device))
    W.pattern_step_grads(model, x, ei, y)
    ref = {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()}
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npz")
        assert set(got.files) == set(ref)
        for n, g in ref.items():
            err = np.abs(got[n] - g).max()
            assert err <= 2e-4 * max(1.0, np.abs(g).max()), (r, n, err, np.abs(g).max())
