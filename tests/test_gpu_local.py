"""Graph-local edge pass (csrc/edge_local.hip): self-contained node windows of a collated batch
(gatx_graph_windows) and the LDS-staged forward edge pass over them (gatx_edge_forward_local),
with the generic pass (gatx_edge_forward_skip) on the remaining nodes. Checked against the
oracle (the reference dataflow, `models/gat_layer.py:42-140`) for concat and head-mean layers,
every fused epilogue, a batch mixing windows with a component too large for one, and — with
attention dropout, whose masks both passes draw from the same counter hash — against the generic
pass itself; bitwise repeatable."""
import numpy as np
import pytest
import torch

from golden_io import grad_seeds
from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4


def _set_local(on):
    """on: True / False forces the graph-local pass on / off; None restores the default (off)."""
    import os
    from gatx.functional import reset_tuning
    if on is None:
        os.environ.pop("GATX_LOCAL", None)
    else:
        os.environ["GATX_LOCAL"] = "1" if on else "0"
    reset_tuning()


def _mixed_batch(sizes, deg=20, fin=24, seed=3):
    """Disjoint graphs of the given node counts (uniform random edges inside each graph)."""
    rng = np.random.default_rng(seed)
    src, dst, off = [], [], 0
    for n in sizes:
        e = n * deg
        src.append(rng.integers(0, n, e) + off)
        dst.append(rng.integers(0, n, e) + off)
        off += n
    ei = np.stack([np.concatenate(src), np.concatenate(dst)]).astype(np.int64)
    x = rng.standard_normal((off, fin)).astype(np.float32)
    return x, ei


def _layer(device, fin, NH, F, concat, bias=False, dropout=0.0, seed=5):
    import gatx
    from gatx import data as gd
    layer = gatx.GATLayer(fin, F, NH, concat, dropout=dropout, add_self_loops=True,
                          bias=bias).to(device)
    W = gd.xavier_uniform(seed, NH * F, fin)
    a = gd.xavier_uniform(seed + 1, NH, NH * 2 * F)
    with torch.no_grad():
        layer.W.weight.copy_(torch.from_numpy(W))
        layer.a.weight.copy_(torch.from_numpy(a))
        if bias:
            layer.bias_param.copy_(torch.linspace(-0.5, 0.5, NH * F))
    return layer, W, a


def test_graph_windows(device):
    """The plan's components are exactly the graphs of the batch, in node order (starts P[0..C],
    P[C] = N); nodes of a component larger than gatx_local_max_nodes are flagged off."""
    import gatx
    from gatx._lib import lib
    T = lib.gatx_local_max_nodes()
    sizes = [300, 1, 2245, T + 50, 17, T]
    x, ei = _mixed_batch(sizes)
    g = gatx.Graph(torch.from_numpy(ei).to(device), x.shape[0], True)
    starts, count, inw = g.window_plan()
    torch.cuda.synchronize()
    offs = np.concatenate([[0], np.cumsum(sizes)])
    C = int(count.item())
    assert C == len(sizes)
    assert np.array_equal(starts.view(-1)[:C + 1].cpu().numpy(), offs)
    flags = np.concatenate([np.full(n, n <= T, dtype=np.uint8) for n in sizes])
    assert np.array_equal(inw[:x.shape[0]].cpu().numpy(), flags)


@pytest.mark.parametrize("NH,F,concat,bias", [(4, 32, True, False), (4, 30, True, True),
                                              (6, 21, False, False), (1, 40, False, True),
                                              (2, 64, True, False)])
def test_local_layer_vs_oracle(NH, F, concat, bias, device):
    """Forward (out, alpha, den through alpha) and backward of a layer on a batch mixing windows
    with a too-large component, against the oracle; the local result equals a second run bitwise
    and the generic pass to fp32 rounding."""
    from gatx._lib import lib
    T = lib.gatx_local_max_nodes()
    # fin = 80: wide enough that no case takes the reassociated (x-row) dataflow
    x, ei = _mixed_batch([500, 1300, T + 100, 64, 1], fin=80)
    layer, W, a = _layer(device, 80, NH, F, concat, bias)
    bias_np = layer.bias_param.detach().cpu().numpy() if bias else None
    r_out, r_ei, r_alpha, cache = orc.gat_layer_forward(x, ei, W, a, NH, F, concat, bias=bias_np)
    res = {}
    try:
        for on in (True, True, False):
            _set_local(on)
            import gatx
            gatx.clear_graph_cache()
            xt = torch.from_numpy(x).to(device).requires_grad_(True)
            out, (ei2, alpha) = layer(xt, torch.from_numpy(ei).to(device),
                                      return_attention_weights=True)
            g_out, _ = grad_seeds(tuple(out.shape), tuple(alpha.shape))
            layer.zero_grad(set_to_none=True)
            (out * torch.from_numpy(g_out).to(device)).sum().backward()
            res.setdefault(on, []).append((out.detach().cpu().numpy(),
                                           alpha.detach().cpu().numpy(),
                                           xt.grad.cpu().numpy(),
                                           layer.W.weight.grad.cpu().numpy()))
            assert np.array_equal(ei2.cpu().numpy(), r_ei)
    finally:
        _set_local(None)
    loc, loc2, gen = res[True][0], res[True][1], res[False][0]
    for u, v in zip(loc, loc2):
        assert np.array_equal(u, v)
    assert np.abs(loc[0] - r_out).max() <= OUT_TOL
    assert np.abs(loc[1] - r_alpha).max() <= OUT_TOL
    g_out, _ = grad_seeds(tuple(r_out.shape), tuple(r_alpha.shape))
    r_g = orc.gat_layer_backward(cache, g_out)
    scale = max(1.0, float(np.abs(r_g["W"]).max()))
    assert np.abs(loc[3] - r_g["W"]).max() <= 1e-4 * scale
    for u, v in zip(loc, gen):
        assert np.abs(u - v).max() <= 1e-5 * max(1.0, float(np.abs(v).max()))


@pytest.mark.parametrize("concat", [True, False])
def test_local_dropout_and_epilogue_match_generic(concat, device):
    """Attention dropout, residual, ELU and the next layer's fused input dropout on the local
    pass give the generic pass's result (same counter-based masks) to fp32 rounding."""
    import gatx
    from gatx.functional import gat_layer_lazy
    x, ei = _mixed_batch([700, 900, 33], fin=40, seed=9)
    NH, F = 4, 16
    layer, W, a = _layer(device, 40, NH, F, concat)
    cols = NH * F if concat else F
    resid = torch.randn(x.shape[0], cols, device=device)
    outs = {}
    try:
        for on in (True, False):
            _set_local(on)
            gatx.clear_graph_cache()
            xt = torch.from_numpy(x).to(device)
            seed = torch.tensor([1234], dtype=torch.int64, device=device)
            oseed = torch.tensor([99], dtype=torch.int64, device=device)
            with torch.no_grad():
                out, _, _ = gat_layer_lazy(
                    xt, torch.from_numpy(ei).to(device), layer.W.weight, layer.a.weight, None,
                    NH, F, concat, True, False, 0.3, seed, resid=resid, elu=True,
                    out_dropout=(0.2, oseed) if concat else None)
            outs[on] = out.cpu().numpy()
    finally:
        _set_local(None)
    assert np.abs(outs[True] - outs[False]).max() <= 1e-5 * max(1.0, np.abs(outs[False]).max())
    assert (outs[True] == 0).sum() == (outs[False] == 0).sum()
