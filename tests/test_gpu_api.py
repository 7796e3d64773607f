"""GPU checks of the layer's API contract beyond numerics: inference_mode, in-place weight updates
that bypass the version counter, and the reference's error behaviour. Compared against the
oracle (`oracle/gat_oracle.py`, pinned to the reference goldens) with the same tolerances as
test_gpu_layer.py."""
import numpy as np
import pytest
import torch

from oracle import gat_oracle as orc

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-4


def _small_case(seed=3, G=2, n=120, e=1500, fin=24, NH=4, F=8):
    from gatx import data as gd
    b = gd.uniform_graph_batch(G, n, e, fin, feature_seed=seed)
    W = gd.xavier_uniform(seed + 1, NH * F, fin)
    a = gd.xavier_uniform(seed + 2, NH, NH * 2 * F)
    return b, W, a, NH, F


def _layer(device, W, a, NH, F, concat=True):
    import gatx
    layer = gatx.GATLayer(W.shape[1], F, NH, concat, add_self_loops=True).to(device)
    with torch.no_grad():
        layer.W.weight.copy_(torch.from_numpy(W))
        layer.a.weight.copy_(torch.from_numpy(a))
    return layer


def test_inference_mode_forward(device):
    """Inference tensors carry no version counter: the graph / weight caches must still key them
    (GraphCache._key read t._version). Model input and edges made in inference mode."""
    import gatx
    from gatx.config import data_config
    b, W, a, NH, F = _small_case()
    layer = _layer(device, W, a, NH, F).eval()
    ref, _, _, _ = orc.gat_layer_forward(b.x, b.edge_index, W, a, NH, F, True)
    with torch.inference_mode():
        x = torch.from_numpy(b.x).to(device)
        ei = torch.from_numpy(b.edge_index).to(device)
        for _ in range(2):   # second call hits the caches
            out = layer(x, ei)
            assert np.abs(out.cpu().numpy() - ref).max() <= OUT_TOL
        model = gatx.GATModel(**data_config["PATTERN"]).to(device).eval()
        xp = torch.randn(b.num_nodes, 3, device=device)
        out = model(xp, ei)
        assert out.shape == (b.num_nodes, 1) and torch.isfinite(out).all()


def test_weight_update_through_data_is_seen(device):
    """`W.data.mul_(2)` does not bump W's version counter. A training forward must use the live
    weights (derived weights are rebuilt whenever gradients flow to them); an eval forward
    after such an update sees it once the cache is cleared."""
    from gatx.functional import clear_weight_cache
    b, W, a, NH, F = _small_case(seed=11)
    layer = _layer(device, W, a, NH, F).train()
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    layer(x, ei).sum().backward()
    v0 = layer.W.weight._version
    layer.W.weight.data.mul_(2.0)
    layer.a.weight.data.mul_(-0.5)
    assert layer.W.weight._version == v0
    out = layer(x, ei)
    ref, _, _, _ = orc.gat_layer_forward(b.x, b.edge_index, 2 * W, -0.5 * a, NH, F, True)
    assert np.abs(out.detach().cpu().numpy() - ref).max() <= OUT_TOL
    layer.eval()
    with torch.no_grad():
        layer(x, ei)                    # caches the current weights
        layer.W.weight.data.mul_(0.5)   # invisible to the version counter ...
        clear_weight_cache()            # ... so the documented remedy
        out = layer(x, ei)
    ref, _, _, _ = orc.gat_layer_forward(b.x, b.edge_index, W, -0.5 * a, NH, F, True)
    assert np.abs(out.cpu().numpy() - ref).max() <= OUT_TOL


@pytest.mark.parametrize("shape", [(4, 8, 24, True), (4, 8, 24, False), (4, 16, 8, True)])
def test_inference_alpha_on_read(shape, device):
    """With `lazy_alpha` set, an inference forward without return_attention_weights defers the
    alpha pass until
    `normalised_attention_coeffs` is read (`models/gat_layer.py:110` stores alpha in every
    forward): the value read is bitwise the eager forward's alpha and matches the oracle, for
    the plain and the reassociated (narrow input) dataflows; a later forward replaces it."""
    NH, F, fin, concat = shape
    b, W, a, _, _ = _small_case(seed=5, fin=fin, NH=NH, F=F)
    layer = _layer(device, W, a, NH, F, concat).eval()
    layer.lazy_alpha = True
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    _, r_ei, r_alpha, _ = orc.gat_layer_forward(b.x, b.edge_index, W, a, NH, F, concat)
    with torch.no_grad():
        out_e, (ei2, alpha_e) = layer(x, ei, return_attention_weights=True)
        alpha_e = alpha_e.clone()
        out_l = layer(x, ei)
        lazy = layer.normalised_attention_coeffs
    assert torch.equal(out_e, out_l)
    assert torch.equal(lazy, alpha_e)
    assert np.array_equal(ei2.cpu().numpy(), r_ei)
    assert np.abs(lazy.cpu().numpy() - r_alpha).max() <= OUT_TOL
    assert layer.normalised_attention_coeffs is lazy   # materialised once
    with torch.no_grad():
        layer(x * 2, ei)
    assert not torch.equal(layer.normalised_attention_coeffs, lazy)


def test_inference_alpha_read_on_another_stream(device):
    """The deferred alpha read from a side stream waits for the forward's stream: bitwise the
    eager alpha, also when the forward was just enqueued behind a long kernel."""
    NH, F, fin = 4, 8, 24
    b, W, a, _, _ = _small_case(seed=6, fin=fin, NH=NH, F=F)
    layer = _layer(device, W, a, NH, F, True).eval()
    layer.lazy_alpha = True
    x = torch.from_numpy(b.x).to(device)
    ei = torch.from_numpy(b.edge_index).to(device)
    with torch.no_grad():
        _, (_, alpha_e) = layer(x, ei, return_attention_weights=True)
        alpha_e = alpha_e.clone()
        big = torch.randn(4096, 4096, device=device)
        torch.cuda.synchronize()
        for _ in range(4):   # keep the forward's stream busy ahead of the forward
            big = big @ big * 1e-3
        layer(x, ei)
    side = torch.cuda.Stream(device)
    with torch.cuda.stream(side):
        lazy = layer.normalised_attention_coeffs.clone()
    side.synchronize()
    assert torch.equal(lazy, alpha_e)
