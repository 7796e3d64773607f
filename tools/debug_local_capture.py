"""Debug: window plan inside a captured hipGraph vs eager (count, flags)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gat-pytorch_amd"))
import torch
import gatx
from gatx import data as gd
from gatx.capture import CapturedStep
dev = torch.device("cuda:0")
b = gd.dataset_batch("PPI", 4)
ei = torch.from_numpy(b.edge_index).to(dev)
N = b.num_nodes
holder = {}

def step():
    gatx.clear_graph_cache()
    g = gatx.graph.graph_cache.get(ei, N, True)
    w, c, inw = g.window_plan()
    holder["t"] = (w, c, inw)
    return c

c0 = step().clone(); torch.cuda.synchronize()
print("eager count", int(c0.item()), "inw sum", int(holder["t"][2][:N].sum().item()))
cap = CapturedStep(step)
w, c, inw = holder["t"]
for i in range(3):
    out = cap(); torch.cuda.synchronize()
    print("replay", i, "count", int(out.item()), "inw sum", int(inw[:N].sum().item()),
          "w0", w[:2].cpu().tolist())
