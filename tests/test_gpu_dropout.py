"""GATModel's input dropout (`models/GATModel.py:130`) on gatx: the standalone kernel
(gatx_dropout) against the oracle's restatement of the counter-based mask, the same dropout fused
into the producing layer's edge-pass epilogue (out_dropout=) against layer-then-kernel, and a
PlanetoidGAT-shaped model in train mode (dropout 0.6: input, inter-layer and attention dropout)
fused vs unfused (gatx.tuning dropout_fuse=0) under the same seeds. torch's own RNG stream cannot be
reproduced bit for bit, so the mask is gatx's (restated in oracle.dropout_keep)."""
import numpy as np
import pytest
import torch

from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,p", [(1000, 37, 0.6), (333, 64, 0.1), (1, 1, 0.5)])
def test_dropout_kernel_vs_oracle_mask(N, C, p, device):
    from gatx.functional import input_dropout
    from gatx import data as gd
    seed = 987654321 + N
    x = torch.from_numpy(gd.normal(N, N * C).reshape(N, C)).to(device).requires_grad_(True)
    y = input_dropout(x, p, seed)
    g = gd.normal(N + 1, N * C).reshape(N, C)
    (y * torch.from_numpy(g).to(device)).sum().backward()
    keep = orc.dropout_keep(seed, N, C, p)
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    ref = np.where(keep, x.detach().cpu().numpy() * scale, np.float32(0))
    np.testing.assert_array_equal(y.detach().cpu().numpy(), ref)
    np.testing.assert_array_equal(x.grad.cpu().numpy(), np.where(keep, g * scale, np.float32(0)))


@pytest.mark.parametrize("fin,NH,F,concat", [(200, 8, 8, True), (64, 8, 3, False),
                                             (64, 6, 124, False), (48, 1, 7, False)])
def test_fused_output_dropout_vs_kernel(fin, NH, F, concat, device):
    """layer(x, elu=True, out_dropout=(p, s)) == gatx_dropout(layer(x, elu=True), p, s): forward
    bit for bit, gradients of x / W / a within fp32 noise (ELU' taken from out * (1 - p))."""
    import gatx
    from gatx import data as gd
    from gatx.functional import fuses_output_dropout, input_dropout
    assert fuses_output_dropout(NH, F, fin, concat)
    b = gd.uniform_graph_batch(2, 180, 2000, fin, feature_seed=51)
    p, s = 0.6, 424242
    res = []
    for fused in (True, False):
        torch.manual_seed(0)
        layer = gatx.GATLayer(fin, F, NH, concat, add_self_loops=True).to(device)
        x = torch.from_numpy(b.x).to(device).requires_grad_(True)
        ei = torch.from_numpy(b.edge_index).to(device)
        if fused:
            out = layer(x, ei, elu=True, out_dropout=(p, s))
        else:
            out = input_dropout(layer(x, ei, elu=True), p, s)
        g = torch.from_numpy(gd.normal(52, out.numel()).reshape(tuple(out.shape))).to(device)
        (out * g).sum().backward()
        res.append((out.detach().cpu().numpy(), x.grad.cpu().numpy(),
                    layer.W.weight.grad.cpu().numpy(), layer.a.weight.grad.cpu().numpy()))
    (o1, *g1), (o0, *g0) = res
    np.testing.assert_array_equal(o1, o0)
    assert (o1 == 0).mean() > 0.4   # the mask is applied
    for a1, a0 in zip(g1, g0):
        assert np.abs(a1 - a0).max() <= 1e-5 * max(1.0, np.abs(a0).max())


@pytest.mark.parametrize("name", ["Cora", "Pubmed"])
def test_planetoid_model_dropout_fused_vs_unfused(name, device, monkeypatch):
    import gatx
    from gatx import data as gd
    from gatx import functional
    from gatx.config import data_config
    cfg = dict(data_config[name])
    # the dataset's layer shapes with a narrower input
    cfg["num_input_node_features"] = 120
    cfg["head_output_features_per_layer"] = [120] + list(cfg["head_output_features_per_layer"][1:])
    b = gd.uniform_graph_batch(1, 700, 5000, cfg["num_input_node_features"], feature_seed=61)
    res = {}
    for fuse in ("1", "0"):
        gatx.tuning.set(dropout_fuse=int(fuse))
        torch.manual_seed(3)
        model = gatx.GATModel(**cfg).to(device).train()
        x = torch.from_numpy(b.x).to(device)
        ei = torch.from_numpy(b.edge_index).to(device)
        out = model(x, ei)
        g = torch.from_numpy(gd.normal(62, out.numel()).reshape(tuple(out.shape))).to(device)
        (out * g).sum().backward()
        res[fuse] = (out.detach().cpu().numpy(),
                     {n: p.grad.cpu().numpy() for n, p in model.named_parameters()})
    (o1, g1), (o0, g0) = res["1"], res["0"]
    assert np.abs(o1 - o0).max() <= 1e-6 * max(1.0, np.abs(o0).max())
    for n in g0:
        assert np.abs(g1[n] - g0[n]).max() <= 1e-5 * max(1.0, np.abs(g0[n]).max()), n
