"""ORACLE-SIDE CPU BASELINE — test/bench infrastructure only (never imported by the product).

The reference GATLayer's forward restated in torch eager, op for op (on CPU for the baseline;
the full-size headline parity test also runs it at fp64 on the device as its checker), so `bench.py`'s
`cpu_baseline` leg times the same ATen dataflow the reference runs on its CPU path
(`cpu_baseline.kind` = "port", the bench contract's word for a restatement of the reference's
algorithm): materialised per-edge gathers with `index_select`, the
(E', NH, 2F) concatenation times `a`, one global `max`, LeakyReLU, `exp`, `scatter_add_` for the
softmax denominators, `index_select` back to edges, the α-weighted messages and a second
`scatter_add_` (`models/gat_layer.py:53-135`, `models/utils.py:6-72`). The reference itself cannot
travel to the GPU box, so this is what is timed there; `bench/cpu_reference_baseline.py` times the
real reference in the build container for comparison.

It is checked against the numpy oracle (`tests/test_oracle_golden.py`), which is pinned to the
reference goldens.
"""
from __future__ import annotations

import torch

LEAKY_SLOPE = 0.01   # nn.LeakyReLU() default (models/gat_layer.py:87)
SOFTMAX_EPS = 1e-8   # models/gat_layer.py:109


def self_loop_rewrite(edge_index: torch.Tensor) -> torch.Tensor:
    """models/utils.py:47-72: drop src == dst, append (i, i) for i <= max id."""
    n = int(edge_index.max()) + 1
    keep = edge_index[0] != edge_index[1]
    loops = torch.arange(n, dtype=edge_index.dtype,
                         device=edge_index.device).unsqueeze(0).expand(2, n)
    return torch.cat([edge_index[:, keep], loops], dim=1)


def _scatter_rows(values: torch.Tensor, index: torch.Tensor, num_rows: int) -> torch.Tensor:
    """scatter_add_ of per-edge rows onto their target nodes (models/utils.py:6-27)."""
    shape = (num_rows,) + tuple(values.shape[1:])
    idx = index.view(-1, *([1] * (values.dim() - 1))).expand_as(values)
    return values.new_zeros(shape).scatter_add_(0, idx, values)


def layer_forward(x, edge_index, W, a, num_heads: int, out_features: int, concat: bool,
                  add_self_loops: bool = True, factorised: bool = False):
    """One GATLayer forward (eval mode, no bias, attention on): returns (out, edge_index', α).
    factorised: the logits as s_src[src] + s_dst[dst] with s = Wh . a's per-side blocks (the same
    sum, SURVEY.md §8a a6, verified to 2e-15 in fp64) instead of the materialised
    (E', NH, 2F) pairs, so autograd through a full-size batch saves no (E', NH, 2F) tensor."""
    NH, F = num_heads, out_features
    if add_self_loops:
        edge_index = self_loop_rewrite(edge_index)
    src, dst = edge_index[0], edge_index[1]
    N = x.size(0)
    Wh = (x @ W.t()).view(N, NH, F)                                   # :64-65
    if factorised:
        A = a.view(NH, NH, 2, F)                                      # a[h, k*2F + s*F + f]
        s_src = torch.einsum("nkf,hkf->nh", Wh, A[:, :, 0, :])
        s_dst = torch.einsum("nkf,hkf->nh", Wh, A[:, :, 1, :])
        raw = s_src.index_select(0, src) + s_dst.index_select(0, dst)
    else:
        pairs = torch.cat([Wh.index_select(0, src), Wh.index_select(0, dst)], dim=-1)  # :70-76
        raw = pairs.view(-1, NH * 2 * F) @ a.t()                      # :76-82, (E', NH)
    t = torch.nn.functional.leaky_relu(raw - raw.max(), LEAKY_SLOPE)   # :84-88
    ex = t.exp()                                                      # :96
    den = _scatter_rows(ex, dst, N)                                   # :97-104
    alpha = ex / (den.index_select(0, dst) + SOFTMAX_EPS)             # :106-110
    msg = Wh.index_select(0, src) * alpha.unsqueeze(-1)               # :117-119
    out = _scatter_rows(msg, dst, N)                                  # :120-127
    out = out.reshape(N, NH * F) if concat else out.mean(dim=1)        # :128-132
    return out, edge_index, alpha


def model_forward(x, edge_index, layers, skips, num_heads, out_features, concat, add_skip,
                  factorised: bool = False):
    """GATModel.forward wiring (models/GATModel.py:120-151) in eval mode: layer -> skip (concat:
    add; mean: add the head-mean of the skip) -> ELU except after the last layer.
    layers: [(W, a)]; skips: per skip-enabled layer, a weight or None (identity)."""
    L = len(layers)
    k = 0
    alphas = []
    ei = edge_index
    for i, (W, a) in enumerate(layers):
        inp = x
        x, ei, alpha = layer_forward(x, ei, W, a, num_heads[i], out_features[i], concat[i],
                                     factorised=factorised)
        alphas.append(alpha)
        if add_skip[i]:
            s = inp if skips[k] is None else inp @ skips[k].t()
            k += 1
            if not concat[i]:
                s = s.view(s.size(0), num_heads[i], out_features[i]).mean(dim=1)
            x = x + s
        if i != L - 1:
            x = torch.nn.functional.elu(x)
    return x, ei, alphas


def attention_norm(edge_index, alphas):
    """GATModel.calc_attention_norm (`models/GATModel.py:189-230`, logging removed) in torch:
    degrees broadcast back to the edges, mean over layers of ||alpha * deg - 1||_1 / E'."""
    dst = edge_index[1]
    E2 = dst.size(0)
    deg = torch.zeros(int(dst.max()) + 1, dtype=alphas[0].dtype).index_add_(
        0, dst, torch.ones(E2, dtype=alphas[0].dtype)).index_select(0, dst)
    norm = 0.0
    for a in alphas:
        norm = norm + (a * deg.unsqueeze(1) - 1.0).abs().sum() / E2
    return norm / len(alphas)
