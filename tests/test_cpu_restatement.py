"""The torch-eager restatement of the reference dataflow (oracle/torch_dataflow.py, bench.py's
cpu_baseline leg) against the numpy oracle, which is pinned to the reference goldens: same
edge_index', alphas and outputs (fp32 noise only) on a PPI-wired 3-layer stack and a PATTERN-wired
4-layer stack with projected skips."""
import numpy as np
import pytest
import torch

from gatx import data as gd
from gatx.config import data_config
from oracle import gat_oracle as orc
from oracle import torch_dataflow as td


@pytest.mark.parametrize("ds,G", [("PPI", 1), ("PATTERN", 4)])
def test_restatement_matches_oracle(ds, G):
    cfg = data_config[ds]
    b = gd.uniform_graph_batch(G, 200 if ds == "PPI" else 119, 3000 if ds == "PPI" else 2000,
                               cfg["num_input_node_features"], graph_seed=9)
    heads = [1] + cfg["num_heads_per_layer"]
    widths = cfg["head_output_features_per_layer"]
    L = cfg["num_layers"]
    layers = [(gd.xavier_uniform(10 + i, heads[i + 1] * widths[i + 1], heads[i] * widths[i]),
               gd.xavier_uniform(20 + i, heads[i + 1], heads[i + 1] * 2 * widths[i + 1]))
              for i in range(L)]
    skips = []
    for i in range(L):
        if cfg["add_skip_connection"][i]:
            fin, fo = heads[i] * widths[i], heads[i + 1] * widths[i + 1]
            skips.append(None if fin == fo else gd.xavier_uniform(30 + i, fo, fin))
    args = (cfg["num_heads_per_layer"], widths[1:], cfg["heads_concat_per_layer"],
            cfg["add_skip_connection"])
    with torch.no_grad():
        out, ei2, al = td.model_forward(
            torch.from_numpy(b.x), torch.from_numpy(b.edge_index),
            [(torch.from_numpy(W), torch.from_numpy(a)) for W, a in layers],
            [None if s is None else torch.from_numpy(s) for s in skips], *args)
    r_out, r_ei, r_al = orc.gat_model_forward(b.x, b.edge_index, layers, skips, *args)
    assert np.array_equal(ei2.numpy(), r_ei)
    scale = max(1.0, float(np.abs(r_out).max()))
    assert np.abs(out.numpy() - r_out).max() <= 1e-4 * scale
    for a, r in zip(al, r_al):
        assert np.abs(a.numpy() - r).max() <= 1e-5


def test_factorised_logits_equal_materialised():
    """torch_dataflow's factorised logits (s_src[src] + s_dst[dst], used by the full-size
    gradient parity test to keep autograd's saved tensors small) equal the reference's
    materialised (E', NH, 2F) . a^T form, forward and gradients, in fp64."""
    import torch
    from oracle import torch_dataflow as td
    g = torch.Generator().manual_seed(4)
    N, E, fin, NH, F = 40, 300, 7, 3, 5
    ei = torch.randint(0, N, (2, E), generator=g)
    outs = []
    for fact in (False, True):
        x = torch.randn(N, fin, generator=torch.Generator().manual_seed(1),
                        dtype=torch.float64).requires_grad_(True)
        W = torch.randn(NH * F, fin, generator=torch.Generator().manual_seed(2),
                        dtype=torch.float64).requires_grad_(True)
        a = torch.randn(NH, NH * 2 * F, generator=torch.Generator().manual_seed(3),
                        dtype=torch.float64).requires_grad_(True)
        out, _, al = td.layer_forward(x, ei, W, a, NH, F, True, factorised=fact)
        (out.sin().sum() + (al * al).sum()).backward()
        outs.append((out.detach(), al.detach(), x.grad, W.grad, a.grad))
    for u, v in zip(*outs):
        assert float((u - v).abs().max()) <= 1e-12 * max(1.0, float(u.abs().max()))
