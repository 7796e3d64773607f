"""Compare the PPI 20-graph forward (edge_lds on) eager vs hipGraph replay vs the L2-gather path,
and time each (diagnostic)."""
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
torch.manual_seed(0)
model = gatx.GATModel(**data_config["PPI"]).to(dev).eval()
b = gd.dataset_batch("PPI", int(sys.argv[1]) if len(sys.argv) > 1 else 20, graph_seed=42,
                     feature_seed=1)
x = torch.from_numpy(b.x).to(dev)
ei = torch.from_numpy(b.edge_index).to(dev)


def step():
    gatx.clear_graph_cache()
    with torch.no_grad():
        return model(x, ei)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


tuning.set(edge_lds=0)
ref = step().clone()
t_ref = timeit(step)
tuning.set(edge_lds=1)
eager = step().clone()
t_eager = timeit(step)
cap = CapturedStep(step)
rep = cap().clone()
t_cap = timeit(cap)
from gatx.graph import graph_cache  # noqa: E402
g = graph_cache.get(ei, b.num_nodes, True)
segs, count = g.node_blocks(2304)
print("blocks", int(count.item()), segs[:int(count.item()) + 1].tolist()[:6])
print(f"gather {t_ref:.3f} ms  lds eager {t_eager:.3f} ms  lds replay {t_cap:.3f} ms")
print("eager vs gather", float((eager - ref).abs().max()))
print("replay vs eager", float((rep - eager).abs().max()))
