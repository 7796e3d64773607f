"""bench.py's exact timed flow (CapturedStep + warmup replays + fallback read + run_timed with its
region marks and instrumented eager steps) with edge_lds on; then checks a replay's output
against the L2-gather path and reads the node-block count the last replay computed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gatx  # noqa: E402
from gatx import _lib, data as gd, tuning  # noqa: E402
from gatx.capture import CapturedStep  # noqa: E402
from gatx.config import data_config  # noqa: E402

dev = torch.device("cuda:0")
tuning.set(edge_lds=1)
torch.manual_seed(0)
model = gatx.GATModel(**data_config["PPI"]).to(dev).eval()
b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
x = torch.from_numpy(b.x).to(dev)
ei = torch.from_numpy(b.edge_index).to(dev)
seen = []


def eager_step():
    gatx.clear_graph_cache()
    with torch.no_grad():
        out = model(x, ei)
    from gatx.graph import graph_cache
    g = graph_cache.get(ei, b.num_nodes, True)
    seen.append(g.node_blocks(2304)[1])
    return out


step = CapturedStep(eager_step)
for _ in range(3):
    step()
fb = torch.zeros(1, dtype=torch.int64, device=dev)
_lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
el, summ, n = bench.run_timed(step, 20, 1, dev, step.eager, False)
print(f"timed {el / 20 * 1e3:.3f} ms")
rep = step().clone()
cnt_replay = int(seen[-1].item()) if seen else None
print("count tensor captured:", seen[1] if len(seen) > 1 else None)
tuning.set(edge_lds=0)
gatx.clear_graph_cache()
with torch.no_grad():
    ref = model(x, ei).clone()
print("replay vs gather", float((rep - ref).abs().max()), "max|ref|", float(ref.abs().max()))
print("counts seen (eager/captured objects):", [int(c.item()) for c in seen])
