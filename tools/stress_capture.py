"""Stress check (diagnostic, not a test): the captured PPI-20 forward (graph build, side-stream
node blocks, LDS-staged pass, side-stream alpha) replayed many times, with a kernel launched
outside the graph before a random subset of replays; every 25th replay's output is compared
with a fresh eager step and the node-block count is read after every replay.
    python tools/stress_capture.py [replays]"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402

import gatx  # noqa: E402
from gatx import data as gd  # noqa: E402
from gatx.capture import CapturedStep  # noqa: E402
from gatx.config import data_config  # noqa: E402
from gatx.graph import graph_cache  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = gatx.GATModel(**data_config["PPI"]).to(dev).eval()
b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
x = torch.from_numpy(b.x).to(dev)
ei = torch.from_numpy(b.edge_index).to(dev)


def step():
    gatx.clear_graph_cache()
    with torch.no_grad():
        return model(x, ei)


ref = step().clone()
cap = CapturedStep(step)
segs, count = graph_cache.get(ei, b.num_nodes, True)._hub_plans[("blocks", 2304)]
rng = random.Random(1)
bad = 0
for i in range(reps):
    if rng.random() < 0.5:
        torch.zeros(rng.randint(1, 4096), device=dev)
    out = cap()
    if i % 25 == 0 or i == reps - 1:
        torch.cuda.synchronize()
        c = int(count.item())
        diff = float((out - ref).abs().max())
        print(f"replay {i}: blocks {c} max|replay - eager| {diff:.3e}", flush=True)
        bad += (c != 20) or diff > 0
torch.cuda.synchronize()
print("stress:", "OK" if bad == 0 else f"{bad} BAD CHECKS")
sys.exit(1 if bad else 0)
