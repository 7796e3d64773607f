"""Hub splitting of the edge passes (gatx_graph_hub_plan + gatx_edge_forward_hubs, and in the
backward gatx_edge_backward_dst_hubs / gatx_edge_backward_src_hubs): destination segments (and,
in the backward's source pass, source segments) longer than gatx.tuning hub_edges are processed in
pieces by parallel waves and combined in piece order. Checked against the oracle (the reference's
dataflow, whose scatter_add_ backward `models/utils.py:17-20` has no per-degree cliff) on graphs
with destination AND source hubs of a few to many pieces, every epilogue kind (concat, one-pass
and multi-pass head mean, the reassociated first layer, dropout), against the unsplit kernels,
and for bitwise repeatability."""
import numpy as np
import pytest
import torch

from golden_io import grad_seeds
from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4
GRAD_TOL = 1e-4


def _hub_graph(n=3000, e=20000, hubs=(30000, 9000, 1001, 1000, 999), fin=16, seed=11,
               src_hubs=(12000, 2500, 1000)):
    """Uniform random edges plus hub destinations receiving the given in-degrees and hub sources
    sending the given out-degrees."""
    rng = np.random.default_rng(seed)
    src = [rng.integers(0, n, e)]
    dst = [rng.integers(0, n, e)]
    for i, d in enumerate(hubs):
        src.append(rng.integers(0, n, d))
        dst.append(np.full(d, 17 + 101 * i))
    for i, d in enumerate(src_hubs):
        src.append(np.full(d, 29 + 97 * i))
        dst.append(rng.integers(0, n, d))
    ei = np.stack([np.concatenate(src), np.concatenate(dst)]).astype(np.int64)
    x = rng.standard_normal((n, fin)).astype(np.float32)
    return x, ei


def _run(device, x, ei, W, a, NH, F, concat, dropout=0.0, grads=True, x_grad=True):
    import gatx
    layer = gatx.GATLayer(x.shape[1], F, NH, concat, dropout=dropout,
                          add_self_loops=True).to(device)
    with torch.no_grad():
        layer.W.weight.copy_(torch.from_numpy(W))
        layer.a.weight.copy_(torch.from_numpy(a))
    if dropout > 0:
        layer._dropout_seed = lambda *_: 77
        layer.train()
    # x_grad=False: the model input (no gradient wanted), which sends a reassociated first
    # layer down _reassoc_backward (gathers over x rows, G_s score rows) instead of layer_backward
    xt = torch.from_numpy(x).to(device).requires_grad_(grads and x_grad)
    et = torch.from_numpy(ei).to(device)
    gatx.clear_graph_cache()
    out, (ei2, alpha) = layer(xt, et, return_attention_weights=True)
    r = dict(out=out.detach().cpu().numpy(), alpha=alpha.detach().cpu().numpy(),
             ei2=ei2.cpu().numpy())
    if grads:
        g_out, g_alpha = grad_seeds(tuple(out.shape), tuple(alpha.shape))
        ((out * torch.from_numpy(g_out).to(device)).sum()
         + (alpha * torch.from_numpy(g_alpha).to(device)).sum()).backward()
        if x_grad:
            r["grad_x"] = xt.grad.cpu().numpy()
        r["grad_W"] = layer.W.weight.grad.cpu().numpy()
        r["grad_a"] = layer.a.weight.grad.cpu().numpy()
    return r


CASES = {   # name: (fin, NH, F, concat, gatx.tuning switches)
    "concat": (16, 4, 16, True, {}),
    "concat_wide": (16, 2, 256, True, {}),
    "mean_one_pass": (16, 6, 12, False, {}),
    "mean_multi_pass": (16, 6, 12, False, {"mean_heads": 2}),
    "reassociated": (8, 4, 64, True, {}),
    "reassociated_input": (8, 4, 64, True, {}),   # x needs no gradient: _reassoc_backward
    "dropout": (16, 4, 16, True, {}),
}


@pytest.mark.parametrize("T", ["1000", "333"])
@pytest.mark.parametrize("name", list(CASES))
def test_hub_split_vs_oracle(name, T, device, monkeypatch):
    fin, NH, F, concat, env = CASES[name]
    dropout = 0.5 if name == "dropout" else 0.0
    from gatx import tuning
    tuning.set(**env)
    tuning.set(hub_edges=int(T), bwd_hub_edges=int(T), hub_min_edges=0)
    from gatx import data as gd
    x, ei = _hub_graph(fin=fin)
    W = gd.xavier_uniform(6, NH * F, fin)
    a = gd.xavier_uniform(7, NH, NH * 2 * F)
    x_grad = name != "reassociated_input"
    keys = ("x", "W", "a") if x_grad else ("W", "a")
    r = _run(device, x, ei, W, a, NH, F, concat, dropout, x_grad=x_grad)
    keep = orc.dropout_keep(77, r["alpha"].shape[0], NH, dropout) if dropout > 0 else None
    out, ei2, alpha, cache = orc.gat_layer_forward(x, ei, W, a, NH, F, concat, dropout_p=dropout,
                                                   keep=keep)
    np.testing.assert_array_equal(r["ei2"], ei2)
    assert np.abs(r["out"] - out).max() <= OUT_TOL
    assert np.abs(r["alpha"] - alpha).max() <= OUT_TOL
    g_out, g_alpha = grad_seeds(out.shape, alpha.shape)
    gr = orc.gat_layer_backward(cache, g_out, g_alpha)
    for k in keys:
        err = np.abs(r[f"grad_{k}"] - gr[k]).max()
        assert err <= GRAD_TOL * max(1.0, np.abs(gr[k]).max()), (k, err)
    # split backward is deterministic: a second run is bitwise identical
    r1 = _run(device, x, ei, W, a, NH, F, concat, dropout, x_grad=x_grad)
    for k in ("out", "alpha") + tuple(f"grad_{k}" for k in keys):
        np.testing.assert_array_equal(r[k], r1[k], err_msg=k)
    # the same layer without splitting: same result to fp32 summation-order noise
    tuning.set(hub_edges=0, bwd_hub_edges=0)
    r0 = _run(device, x, ei, W, a, NH, F, concat, dropout, x_grad=x_grad)
    assert np.abs(r["out"] - r0["out"]).max() <= 1e-5
    assert np.abs(r["alpha"] - r0["alpha"]).max() <= 1e-5
    for k in keys:
        err = np.abs(r[f"grad_{k}"] - r0[f"grad_{k}"]).max()
        assert err <= 1e-5 * max(1.0, np.abs(r0[f"grad_{k}"]).max()), (k, err)


def test_hub_plan(device, monkeypatch):
    """The plan lists every segment longer than T as ceil(deg / T) pieces in consecutive slots."""
    from gatx import clear_graph_cache
    from gatx.graph import graph_cache
    x, ei = _hub_graph()
    clear_graph_cache()
    g = graph_cache.get(torch.from_numpy(ei).to(device), x.shape[0], True)
    hubs, count, bound = g.hub_plan(1000)
    torch.cuda.synchronize()
    rowptr = g.rowptr.cpu().numpy()
    deg = np.diff(rowptr)
    want = {int(n): int(-(-d // 1000)) for n, d in enumerate(deg) if d > 1000}
    c = int(count.item())
    h = hubs[:c].cpu().numpy()
    assert c == sum(want.values()) and c <= bound
    got = {}
    for node, p, pieces, first in h:
        assert want[int(node)] == pieces
        got.setdefault(int(node), set()).add((int(p), int(first)))
    for node, pcs in got.items():
        firsts = {f for _, f in pcs}
        assert len(firsts) == 1 and {p for p, _ in pcs} == set(range(want[node]))
    # slot ranges of different hubs are disjoint and cover [0, count)
    starts = sorted((f, want[n]) for n, pcs in got.items() for f in {f for _, f in pcs})
    pos = 0
    for f, pieces in starts:
        assert f == pos
        pos += pieces
    assert pos == c


def test_source_hub_plan(device):
    """The backward's source-side plan lists the transpose's long segments (source hubs)."""
    from gatx import clear_graph_cache
    from gatx.graph import graph_cache
    x, ei = _hub_graph()
    clear_graph_cache()
    g = graph_cache.get(torch.from_numpy(ei).to(device), x.shape[0], True)
    hubs, count, bound = g.hub_plan(1000, source=True)
    torch.cuda.synchronize()
    deg = np.diff(g.srowptr.cpu().numpy())
    want = {int(n): int(-(-d // 1000)) for n, d in enumerate(deg) if d > 1000}
    assert {29: 13, 126: 3}.items() <= want.items()
    c = int(count.item())
    h = hubs[:c].cpu().numpy()
    assert c == sum(want.values())
    assert {int(node): int(pieces) for node, _, pieces, _ in h} == want


def test_rmat_scaled_backward_hub_split(device, monkeypatch):
    """A scaled R-MAT graph (1e6 nodes, 1.6e7 edges: past the 2^22-edge threshold, so the
    default plan splits every segment longer than 8192 edges) through forward + backward: the
    hub-split backward passes give the unsplit passes' gradients to fp32 summation noise, and
    the plan really has destination and source hubs."""
    import gatx
    from gatx import data as gd
    from gatx.graph import graph_cache
    N, E, NH, F, FIN = 1_000_000, 16_000_000, 8, 64, 64
    ei = gd.rmat_edges_device(N, E, seed=5, device=device)
    torch.manual_seed(0)
    layer = gatx.GATLayer(FIN, F, NH, True, add_self_loops=True).to(device)
    g = torch.Generator(device=device)
    g.manual_seed(2)
    x0 = torch.randn(N, FIN, device=device, generator=g)
    gout = torch.randn(N, NH * F, device=device, generator=g)

    from gatx import tuning
    tuning.set(bwd_hub_edges=8192)   # split at the forward's threshold

    def run(split):
        tuning.set(bwd_hubs=1 if split else 0)
        gatx.clear_graph_cache()
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        layer(x, ei).backward(gout)
        torch.cuda.synchronize()
        return x.grad, layer.W.weight.grad.clone(), layer.a.weight.grad.clone()

    split = run(True)
    graph = graph_cache.get(ei, N, True)
    d_hubs = int(graph.hub_plan(8192)[1].item())
    s_hubs = int(graph.hub_plan(8192, source=True)[1].item())
    assert d_hubs > 0 and s_hubs > 0, (d_hubs, s_hubs)
    again = run(True)
    for a_, b_ in zip(split, again):
        assert torch.equal(a_, b_)   # bitwise repeatable
    plain = run(False)
    for name, a_, b_ in zip(("x", "W", "a"), split, plain):
        scale = max(1.0, float(b_.abs().max()))
        err = float((a_ - b_).abs().max())
        assert err <= 1e-5 * scale, (name, err, scale)
