"""GATModel's Linear skip folded into the layer's projection GEMM (GATLayer(..., skip_weight=W_s):
W_s's rows appended to W_aug, the skip output written as the GEMM's third output range and added
by the edge-pass / output-projection epilogue) against the fp64 oracle: the layer plus
`x W_s^T` (concat) or its head mean (`models/GATModel.py:136-145`), ELU, and the gradients of x,
W, a and W_s. Covers both first-layer dataflows (reassociated: the skip rides on the score GEMM;
direct: gatx_projection_gemm3), head mean, const attention and an input without gradient.
Model level: a PATTERN-shaped GATModel (every layer a Linear skip) with the fold matches the
oracle's model forward/backward and the unfolded path (gatx.tuning skip_fold=0)."""
import numpy as np
import pytest

DEFAULT_GEMM_MODE = 2   # f16x3 (csrc/gemm.hip gemm_mode)
import torch

from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4
GRAD_TOL = 1e-4


def _skip_ref(x, Ws, NH, F, concat):
    so = x @ Ws.T
    return so if concat else so.reshape(-1, NH, F).mean(axis=1)


@pytest.mark.parametrize("fin,NH,F,concat,const,elu,need_x", [
    (3, 4, 12, True, False, True, False),     # PATTERN L0: reassociated, input without grad
    (48, 4, 24, True, False, True, True),     # PATTERN L1: reassociated, general backward
    (96, 4, 12, True, False, True, True),     # PATTERN L2: direct projection (gemm3)
    (48, 1, 1, False, False, False, True),    # PATTERN L3: one-head mean, no ELU
    (32, 4, 16, False, False, True, True),    # head mean over 4 heads
    (64, 6, 37, False, False, False, True),   # head mean, F % 4 != 0
    (96, 4, 12, True, True, True, True),      # const attention, direct
    (5, 4, 12, True, True, False, False),     # const attention, reassociated
])
def test_folded_skip_layer_vs_oracle(fin, NH, F, concat, const, elu, need_x, device):
    _check_folded_skip_layer(fin, NH, F, concat, const, elu, need_x, device, 150, 1800)


def test_folded_skip_reassoc_large(device):
    """The all-skip PPI variant's first layer (50 -> 4 x 256, reassociated, no input gradient)
    at a size where the skip weight's gradient GEMM reads go directly (N C >= 2^22) instead of a
    copy in G_s (functional._reassoc_backward skip_from_go)."""
    _check_folded_skip_layer(50, 4, 256, True, False, True, False, device, 1400, 12000)


def _check_folded_skip_layer(fin, NH, F, concat, const, elu, need_x, device, nodes, edges):
    import gatx
    from gatx import data as gd
    b = gd.uniform_graph_batch(3, nodes, edges, fin, feature_seed=31 + fin)
    W = gd.xavier_uniform(32 + NH, NH * F, fin)
    a = gd.xavier_uniform(33 + NH, NH, NH * 2 * F)
    Ws = gd.xavier_uniform(34 + F, NH * F, fin)
    layer = gatx.GATLayer(fin, F, NH, concat, add_self_loops=True,
                          const_attention=const).to(device)
    with torch.no_grad():
        layer.W.weight.copy_(torch.from_numpy(W))
        if not const:
            layer.a.weight.copy_(torch.from_numpy(a))
    x = torch.from_numpy(b.x).to(device).requires_grad_(need_x)
    ws = torch.from_numpy(Ws).to(device).requires_grad_(True)
    ei = torch.from_numpy(b.edge_index).to(device)
    out = layer(x, ei, skip_weight=ws, elu=elu)
    g = gd.normal(35, out.numel()).reshape(tuple(out.shape))
    (out * torch.from_numpy(g).to(device)).sum().backward()
    torch.cuda.synchronize()

    xd = b.x.astype(np.float64)
    o, _, _, cache = orc.gat_layer_forward(xd, b.edge_index, W, a, NH, F, concat,
                                           const_attention=const, dtype=np.float64)
    pre = o + _skip_ref(xd, Ws.astype(np.float64), NH, F, concat)
    post = orc.elu(pre) if elu else pre
    assert np.abs(out.detach().cpu().numpy() - post).max() <= OUT_TOL
    g_pre = g * np.where(pre > 0, 1.0, np.exp(np.minimum(pre, 0))) if elu else g.astype(np.float64)
    gr = orc.gat_layer_backward(cache, g_pre)
    g_so = g_pre if concat else np.repeat(g_pre[:, None, :] / NH, NH, axis=1).reshape(len(xd), -1)
    refs = [("W", layer.W.weight.grad, gr["W"]), ("skip", ws.grad, g_so.T @ xd)]
    if not const:
        refs.append(("a", layer.a.weight.grad, gr["a"]))
    if need_x:
        refs.append(("x", x.grad, gr["x"] + g_so @ Ws.astype(np.float64)))
    else:
        assert x.grad is None
    for k, t, ref in refs:
        err = np.abs(t.cpu().numpy() - ref).max()
        assert err <= GRAD_TOL * max(1.0, np.abs(ref).max()), (k, err)


def _pattern_model(device, seed):
    import gatx
    from gatx.config import data_config
    torch.manual_seed(seed)
    return gatx.GATModel(**data_config["PATTERN"]).to(device)


def test_folded_skip_pattern_model(device, monkeypatch):
    """PATTERN 4-layer model (Linear skips on every layer, 3 -> 48 -> 96 -> 48 -> 1): folded
    forward and gradients vs the fp64 oracle, and vs the unfolded path within fp32 noise."""
    from gatx import data as gd
    from gatx.config import data_config
    cfg = data_config["PATTERN"]
    b = gd.uniform_graph_batch(4, 120, 1400, cfg["num_input_node_features"], feature_seed=41)
    ei = torch.from_numpy(b.edge_index).to(device)
    results = {}
    for fold in ("1", "0"):
        from gatx import tuning
        tuning.set(skip_fold=int(fold))
        model = _pattern_model(device, 5)
        x = torch.from_numpy(b.x).to(device)
        out = model(x, ei)
        g = torch.from_numpy(gd.normal(42, out.numel()).reshape(tuple(out.shape))).to(device)
        (out * g).sum().backward()
        torch.cuda.synchronize()
        results[fold] = (out.detach().cpu().numpy(),
                         {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters()},
                         model, g.cpu().numpy())
    out1, gr1, model, g = results["1"]
    out0, gr0, _, _ = results["0"]
    for n in gr1:
        assert np.abs(gr1[n] - gr0[n]).max() <= 1e-4 * max(1.0, np.abs(gr0[n]).max()), n
    assert np.abs(out1 - out0).max() <= 1e-4
    L = cfg["num_layers"]
    layers = [(model.gat_layer_list[i].W.weight.detach().cpu().numpy(),
               model.gat_layer_list[i].a.weight.detach().cpu().numpy()) for i in range(L)]
    skips = [s.weight.detach().cpu().numpy() for s in model.skip_layer_list]
    ref_out, ref = orc.gat_model_forward_backward(
        b.x, b.edge_index, layers, skips, cfg["num_heads_per_layer"],
        cfg["head_output_features_per_layer"][1:], cfg["heads_concat_per_layer"],
        cfg["add_skip_connection"], g)
    scale = max(1.0, np.abs(ref_out).max())
    assert np.abs(out1 - ref_out).max() <= OUT_TOL * scale
    for i in range(L):
        for k, name in (("W", f"gat_layer_list.{i}.W.weight"), ("a", f"gat_layer_list.{i}.a.weight"),
                        ("skip", f"skip_layer_list.{i}.weight")):
            r = ref[k][i]
            assert np.abs(gr1[name] - r).max() <= GRAD_TOL * max(1.0, np.abs(r).max()), name


@pytest.mark.parametrize("ds", ["PPI", "PATTERN"])
def test_reference_wiring_equals_fused(ds, device):
    """gatx.GATModel with fuse_wiring=False runs the reference's GATModel.forward op for op
    around gatx layers (the INTEGRATION.md drop-in; bench.py --wiring reference): same output
    and gradients as the fused wiring within fp32 noise."""
    import gatx
    from gatx import data as gd
    from gatx.config import data_config
    cfg = dict(data_config[ds])
    b = gd.dataset_batch(ds, 2, graph_seed=7, feature_seed=8)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    res = []
    for fuse in (True, False):
        torch.manual_seed(11)
        model = gatx.GATModel(**cfg).to(device)
        model.fuse_wiring = fuse
        out = model(x, ei)
        g = torch.from_numpy(gd.normal(9, out.numel()).reshape(tuple(out.shape))).to(device)
        (out * g).sum().backward()
        res.append((out.detach().cpu().numpy(),
                    {n: p.grad.cpu().numpy() for n, p in model.named_parameters()}))
    (o1, g1), (o0, g0) = res
    assert np.abs(o1 - o0).max() <= 1e-4 * max(1.0, np.abs(o0).max())
    for n in g0:
        assert np.abs(g1[n] - g0[n]).max() <= 1e-4 * max(1.0, np.abs(g0[n]).max()), n


def test_model_accepts_reference_data_object(device):
    """forward(data) / forward_and_return_attention(data) as the reference calls them
    (`models/GATModel.py:120-121, 153-154`: data.x, data.edge_index)."""
    from types import SimpleNamespace
    import gatx
    from gatx import data as gd
    from gatx.config import data_config
    b = gd.dataset_batch("PATTERN", 2, graph_seed=3, feature_seed=4)
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    torch.manual_seed(2)
    model = gatx.GATModel(**data_config["PATTERN"]).to(device).eval()
    data = SimpleNamespace(x=x, edge_index=ei)
    with torch.no_grad():
        a = model(x, ei)
        b2 = model(data)
        o, ei2, atts = model.forward_and_return_attention(data)
    assert torch.equal(a, b2) and torch.equal(a, o)
    assert len(atts) == data_config["PATTERN"]["num_layers"] and ei2.shape[0] == 2


@pytest.mark.parametrize("mode", [2, 1, 0])   # f16x3 (default), x3 and f32-MFMA arithmetic
@pytest.mark.parametrize("M,N,K,s1,s2", [(96, 300, 64, 128, 200), (44900, 1036 + 48, 256, 1024, 1036),
                                          (3001, 450, 96, 48, 56)])
def test_projection_gemm3_three_outputs(mode, M, N, K, s1, s2, device):
    """gatx_projection_gemm3's three output ranges (the folded skip's C2) in both arithmetics,
    including shapes whose last partial wave is split along K (workspace, fix-up kernel)."""
    from gatx._lib import call, lib, ptr, stream
    from gatx.functional import gemm_workspace
    g = torch.Generator(device=device).manual_seed(M + N)
    A = torch.randn(M, K, device=device, generator=g)
    W = torch.randn(N, K, device=device, generator=g)   # B(k, n) = W[n, k], as W_aug
    C0 = torch.full((M, s1), float("nan"), device=device)
    C1 = torch.full((M, s2 - s1), float("nan"), device=device)
    C2 = torch.full((M, N - s2), float("nan"), device=device)
    lib.gatx_set_gemm_mode(mode)
    try:
        ws = gemm_workspace(M, N, K, device)
        call("gatx_projection_gemm3", M, N, K, ptr(A), K, 1, ptr(W), 1, K, ptr(C0), s1, s1,
             ptr(C1), s2 - s1, s2, ptr(C2), N - s2, *ws, stream())
        torch.cuda.synchronize()
    finally:
        lib.gatx_set_gemm_mode(DEFAULT_GEMM_MODE)
    ref = A.double() @ W.double().t()
    got = torch.cat([C0, C1, C2], 1).double()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 1e-4 * max(1.0, K ** 0.5)
