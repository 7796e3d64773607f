"""Child process of tests/test_gpu_distributed.py: one rank of PATTERN graph-batch data-parallel
training (BASELINE config 4, `models/pattern_gat.py:18-25`) through gatx.GATModel on cuda:0. Rank
r takes graphs r::world of a fixed 8-graph batch (uneven for world 3), scales each mean loss term
by its count weight (nodes for the BCE, edges E' for the attention norm, count_weights), and the
overlapped GradientAllReducer SUMs the gradients. Writes the reduced gradients to
<out_dir>/rank<r>.npz.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python dist_pattern_worker.py OUT_DIR [gloo|nccl] [bce|bce+norm]

gloo is the stand-in for RCCL when several ranks share one GPU. `nccl` (RCCL) runs at world size
1 on a one-GPU box, with the reducer and count_weights forced through their collectives
(always_reduce), so the device-tensor async all-reduce path runs on hardware.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-pytorch_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gatx import GATModel  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx.config import data_config  # noqa: E402
from gatx.distributed import GradientAllReducer, collate_graphs, count_weights, shard_graphs  # noqa: E402
from gatx.graph import graph_cache  # noqa: E402

NUM_GRAPHS = 8
NORM_WEIGHT = 0.5   # attention_penalty-style weight of calc_attention_norm in "bce+norm"


def pattern_graphs(device):
    """8 PATTERN-shaped graphs (119 nodes, 6099 edges each) with binary node labels."""
    b = gd.dataset_batch("PATTERN", NUM_GRAPHS, graph_seed=314, feature_seed=15)
    y = (gd.uniform01(27, b.num_nodes) < 0.1765).astype(np.float32)
    out = []
    for g in range(NUM_GRAPHS):
        n0, n1 = int(b.node_offsets[g]), int(b.node_offsets[g + 1])
        m = (b.edge_index[1] >= n0) & (b.edge_index[1] < n1)
        out.append((torch.from_numpy(b.x[n0:n1]).to(device),
                    torch.from_numpy(b.edge_index[:, m] - n0).to(device),
                    torch.from_numpy(y[n0:n1]).to(device)))
    return out


def pattern_step_grads(model, x, ei, y, weight=1.0, loss="bce", w_edges=1.0):
    """PatternGAT.training_step (models/pattern_gat.py:18-25): class-balanced BCE mean; with
    loss "bce+norm" plus NORM_WEIGHT x calc_attention_norm (the PPI_GAT attention_penalty term,
    models/ppi_gat.py:22-33, a per-edge mean)."""
    loss_fn = torch.nn.BCEWithLogitsLoss(
        pos_weight=torch.tensor([1 / 0.1765], device=x.device))
    if loss == "bce":
        out = model(x, ei).squeeze(-1)
        (loss_fn(out, y) * weight).backward()
        return
    out, ei2, atts = model.forward_and_return_attention(x, ei)
    norm = model.calc_attention_norm(ei2, atts)
    (loss_fn(out.squeeze(-1), y) * weight + NORM_WEIGHT * w_edges * norm).backward()


def main():
    out_dir = sys.argv[1]
    backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
    loss = sys.argv[3] if len(sys.argv) > 3 else "bce"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    force = backend == "nccl"
    torch.manual_seed(0)
    model = GATModel(**data_config["PATTERN"]).to(dev).train()
    reducer = GradientAllReducer(model.parameters(), average=False, always_reduce=force)
    assert reducer.active
    graphs = pattern_graphs(dev)
    x, ei, y, _ = collate_graphs([graphs[i] for i in shard_graphs(NUM_GRAPHS, rank, world)])
    e_local = graph_cache.get(ei, x.size(0), True).num_edges
    w_n, w_e = count_weights([x.size(0), e_local], device=dev if force else "cpu",
                             always_reduce=force)
    model.zero_grad(set_to_none=True)
    pattern_step_grads(model, x, ei, y, w_n, loss, w_e)
    reducer.finish()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"),
             **{n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
