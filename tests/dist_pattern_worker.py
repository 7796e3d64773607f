"""Child process of tests/test_gpu_distributed.py: one rank of PATTERN graph-batch data-parallel
training (BASELINE config 4, `models/pattern_gat.py:18-25`) through gatx.GATModel on cuda:0, over
gloo (the test-only stand-in for RCCL when both ranks share one GPU). Rank r takes graphs r::world
of a fixed 8-graph batch, scales its mean loss by count_weight(n_local), and the overlapped
GradientAllReducer SUMs the gradients. Writes the reduced gradients to <out_dir>/rank<r>.npz.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dist_pattern_worker.py OUT_DIR
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
from gatx.distributed import GradientAllReducer, collate_graphs, count_weight, shard_graphs  # noqa: E402

NUM_GRAPHS = 8


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


def pattern_step_grads(model, x, ei, y, weight=1.0):
    """PatternGAT.training_step (models/pattern_gat.py:18-25): class-balanced BCE mean."""
    loss_fn = torch.nn.BCEWithLogitsLoss(
        pos_weight=torch.tensor([1 / 0.1765], device=x.device))
    out = model(x, ei).squeeze(-1)
    (loss_fn(out, y) * weight).backward()


def main():
    out_dir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    model = GATModel(**data_config["PATTERN"]).to(dev).train()
    reducer = GradientAllReducer(model.parameters(), average=False)
    graphs = pattern_graphs(dev)
    x, ei, y, _ = collate_graphs([graphs[i] for i in shard_graphs(NUM_GRAPHS, rank, world)])
    w = count_weight(x.size(0))
    model.zero_grad(set_to_none=True)
    pattern_step_grads(model, x, ei, y, w)
    reducer.finish()
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"),
             **{n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
