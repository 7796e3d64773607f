"""Time the REAL reference GATLayer (imported read-only from /root/reference) on this container's
CPU cores, at the BASELINE / SURVEY.md §8(d) uniform-graph configs; writes
bench/cpu_reference_baseline.json. Build-container only (the reference never travels to the GPU
box); the GPU box times oracle/torch_dataflow.py, the same ATen dataflow, as bench.py's
cpu_baseline. The 3-layer PPI / 4-layer PATTERN stacks are wired exactly as
models/GATModel.py:120-151 (GATModel itself needs pytorch_lightning, absent here), eval mode,
torch.no_grad(), 1 warm-up, min of >= 3 reps.

    PYTHONDONTWRITEBYTECODE=1 python bench/cpu_reference_baseline.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(ROOT, "gat-pytorch_amd"))
sys.path.insert(0, "/root/reference")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from models.gat_layer import GATLayer  # noqa: E402  (reference, read-only)

from gatx import data as gd  # noqa: E402
from gatx.config import data_config  # noqa: E402


def build_stack(cfg):
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    layers, skips = [], []
    for i in range(cfg["num_layers"]):
        fin = heads[i] * widths[i]
        layers.append(GATLayer(fin, widths[i + 1], heads[i + 1], cfg["heads_concat_per_layer"][i],
                               dropout=cfg["dropout"], add_self_loops=True, bias=False).eval())
        if cfg["add_skip_connection"][i]:
            out = heads[i + 1] * widths[i + 1]
            skips.append(torch.nn.Identity() if fin == out
                         else torch.nn.Linear(fin, out, bias=False))
    return layers, skips, heads, widths


def stack_forward(cfg, layers, skips, heads, widths, x, ei):
    """models/GATModel.py:120-151 in eval mode."""
    k = 0
    L = len(layers)
    for i in range(L):
        inp = x
        x = layers[i](x, ei)
        if cfg["add_skip_connection"][i]:
            s = skips[k](inp)
            k += 1
            if cfg["heads_concat_per_layer"][i]:
                x = x + s
            else:
                x = x + s.view(-1, heads[i + 1], widths[i + 1]).mean(dim=1)
        if i != L - 1:
            x = F.elu(x)
    return x


def time_it(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    res = {"source": "reference models/gat_layer.py imported from /root/reference (read-only), "
                     "torch " + torch.__version__ + " CPU",
           "cores": cores, "torch_threads": torch.get_num_threads(), "unit": "layer-edges/s",
           "configs": {}}
    for name, ds, G in [("PPI 3-layer fwd, G=1", "PPI", 1), ("PPI 3-layer fwd, G=2", "PPI", 2),
                        ("PATTERN 4-layer fwd, G=8", "PATTERN", 8)]:
        cfg = data_config[ds]
        b = gd.dataset_batch(ds, G, graph_seed=4242)
        x = torch.from_numpy(b.x)
        ei = torch.from_numpy(b.edge_index)
        layers, skips, heads, widths = build_stack(cfg)
        with torch.no_grad():
            t = time_it(lambda: stack_forward(cfg, layers, skips, heads, widths, x, ei))
            _, (ei2, _) = layers[0](x, ei, return_attention_weights=True)
        le = cfg["num_layers"] * ei2.shape[1]
        res["configs"][name] = {"nodes": b.num_nodes, "edges_per_layer": int(ei2.shape[1]),
                                "seconds": t, "value": le / t}
        print(name, round(t, 3), "s", round(le / t / 1e6, 3), "M layer-edges/s", flush=True)
    # Cora single layer (BASELINE config 2 shape): 1433 -> 8 x 8 concat
    b = gd.dataset_batch("Cora", 1, graph_seed=4242)
    lay = GATLayer(1433, 8, 8, True, add_self_loops=True).eval()
    x = torch.from_numpy(b.x)
    ei = torch.from_numpy(b.edge_index)
    with torch.no_grad():
        t = time_it(lambda: lay(x, ei))
        _, (ei2, _) = lay(x, ei, return_attention_weights=True)
    res["configs"]["Cora GATLayer fwd (1433 -> 8x8)"] = {
        "nodes": b.num_nodes, "edges_per_layer": int(ei2.shape[1]), "seconds": t,
        "value": ei2.shape[1] / t}
    print("Cora", round(t, 4), "s", flush=True)
    out = os.path.join(ROOT, "bench", "cpu_reference_baseline.json")
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
