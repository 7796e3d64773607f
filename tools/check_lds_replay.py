"""Diagnostic: which host action between a captured LDS-path forward's replays makes later replays
skip the LDS-staged edge pass (bench.py's timed replays ran edge_lds_kernel in ~6.5 us after the
fallback-counter read). Replays the captured PPI forward, timing each replay with HIP events, and
between replay 3 and 4 performs the action named by argv[1]:
  none | zeros (a 1-element torch.zeros) | fbread (zeros + gatx_gemm_fallback_read) |
  sync (torch.cuda.synchronize only) | mark (gatx_region_mark)
Prints per-replay ms and the capture-time graph's node-block count / first bounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]
import torch  # noqa: E402

import gatx  # noqa: E402
from gatx import _lib, data as gd, tuning  # noqa: E402
from gatx.capture import CapturedStep  # noqa: E402
from gatx.config import data_config  # noqa: E402
from gatx.graph import graph_cache  # noqa: E402

action = sys.argv[1] if len(sys.argv) > 1 else "none"
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
g = graph_cache._cache if hasattr(graph_cache, "_cache") else None
gobj = graph_cache.get(ei, b.num_nodes, True)   # the capture-time graph (still cached)
segs, count = gobj._hub_plans[("blocks", 2304)]


def state():
    torch.cuda.synchronize()
    return int(count.item()), segs[:3].tolist()


times = []
for i in range(8):
    if i == 4:
        torch.cuda.synchronize()
        if action in ("zeros", "fbread"):
            fb = torch.zeros(1, dtype=torch.int64, device=dev)
            if action == "fbread":
                _lib.call("gatx_gemm_fallback_read", _lib.ptr(fb), 1, _lib.stream())
        elif action == "mark":
            _lib.call("gatx_region_mark", 8, _lib.stream())
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = cap()
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1))
    print(f"{action} replay {i}: {times[-1]:.3f} ms  blocks {state()}", flush=True)
rep = out.clone()
tuning.set(edge_lds=0)
ref = step().clone()
print(f"{action}: replay vs gather {float((rep - ref).abs().max()):.3e}")
