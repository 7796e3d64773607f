"""bench.py's flow with edge_lds on from the start (CapturedStep built before any eager step):
replay output vs the L2-gather path, and replay time (diagnostic)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402

import gatx  # noqa: E402
from gatx import data as gd, tuning  # noqa: E402
from gatx.capture import CapturedStep  # noqa: E402
from gatx.config import data_config  # noqa: E402

dev = torch.device("cuda:0")
tuning.set(edge_lds=1)
torch.manual_seed(0)
model = gatx.GATModel(**data_config["PPI"]).to(dev).eval()
b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
x = torch.from_numpy(b.x).to(dev)
ei = torch.from_numpy(b.edge_index).to(dev)


def step():
    gatx.clear_graph_cache()
    with torch.no_grad():
        return model(x, ei)


cap = CapturedStep(step)
for _ in range(2):
    cap()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    out = cap()
torch.cuda.synchronize()
print(f"replay {(time.perf_counter() - t) / 20 * 1e3:.3f} ms")
rep = out.clone()
eag = cap.eager().clone()
tuning.set(edge_lds=0)
ref = step().clone()
print("replay vs eager(lds)", float((rep - eag).abs().max()))
print("replay vs gather", float((rep - ref).abs().max()), "max|ref|", float(ref.abs().max()))
