"""A/B of functional._reassoc_backward's skip_from_go on the all-skip PPI variant
(config.NOTEBOOK_VARIANTS, the bench's 20 graphs): one training step (forward + backward) timed with HIP events,
interleaved on and off, 200 steps each."""
import sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gat-pytorch_amd")]
import torch
import gatx
from gatx import data as gd, functional
from gatx.config import data_config, NOTEBOOK_VARIANTS

dev = torch.device("cuda:0")
cfg = dict(data_config["PPI"]); cfg.update(add_skip_connection=NOTEBOOK_VARIANTS["PPI"]["add_skip_connection"])
torch.manual_seed(0)
model = gatx.GATModel(**cfg).to(dev).train()
b = gd.dataset_batch("PPI", 20, graph_seed=42, feature_seed=1)
x = torch.from_numpy(b.x).to(dev); ei = torch.from_numpy(b.edge_index).to(dev)
g = torch.randn(x.size(0), cfg["num_classes"], device=dev)


def step():
    out = model(x, ei)
    (out * g).sum().backward()


res = {"on": [], "off": []}
for rnd in range(10):
    for mode in ("on", "off"):
        functional.SKIP_FROM_GO_MIN = (1 << 22) if mode == "on" else (1 << 62)
        for _ in range(3):
            step()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); s.record()
        for _ in range(20):
            step()
        e.record(); torch.cuda.synchronize()
        res[mode].append(s.elapsed_time(e) / 20)
for m, v in res.items():
    v = sorted(v)
    print(m, "median ms/step", round(v[len(v) // 2], 4), "min", round(v[0], 4))
