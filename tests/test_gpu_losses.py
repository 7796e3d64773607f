"""gatx.losses.bce_with_logits (csrc/loss.hip) against torch's binary_cross_entropy_with_logits —
the task modules' loss (PPI_GAT `models/ppi_gat.py:11,19`; PatternGAT with pos_weight
`models/pattern_gat.py:11-15`): loss value and input gradient, one-launch and two-launch sizes,
extreme logits, bitwise repeatability."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 952, 65536, 65537, 44900 * 121])
@pytest.mark.parametrize("pw", [None, 1 / 0.1765])
def test_bce_matches_torch(n, pw, device):
    from gatx.losses import bce_with_logits
    g = torch.Generator(device=device).manual_seed(n)
    x = (torch.randn(n, device=device, generator=g) * 6).requires_grad_(True)
    x.data[: min(n, 4)] = torch.tensor([80.0, -80.0, 0.0, 1e-3], device=device)[: min(n, 4)]
    y = (torch.rand(n, device=device, generator=g) > 0.5).float()
    pwt = None if pw is None else torch.tensor([pw], device=device)
    ref = torch.nn.functional.binary_cross_entropy_with_logits(x.double(), y.double(),
                                                               pos_weight=pwt and pwt.double())
    gref, = torch.autograd.grad(ref, x)
    x2 = x.detach().clone().requires_grad_(True)
    got = bce_with_logits(x2, y, pw)
    (got * 3.0).backward()
    assert abs(got.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    err = (x2.grad.double() - 3.0 * gref).abs().max().item()
    assert err <= 1e-6 * max(1.0, (3.0 * gref).abs().max().item()) + 1e-9, err
    # fixed-order reductions: a second evaluation is bitwise identical
    again = bce_with_logits(x2.detach(), y, pw)
    assert again.item() == got.item()


def test_bce_module_and_shape_check(device):
    from gatx.losses import BCEWithLogitsLoss
    loss = BCEWithLogitsLoss(pos_weight=torch.tensor([2.0]))
    x = torch.zeros(3, 4, device=device)
    assert abs(loss(x, torch.ones(3, 4, device=device)).item() - 2.0 * 0.6931471805599453) < 1e-6
    with pytest.raises(ValueError):
        loss(x, torch.ones(4, 3, device=device))
    # a target that wants a gradient is refused (torch would differentiate it; the fused kernel
    # only writes the input's gradient)
    with pytest.raises(RuntimeError, match="target"):
        loss(x, torch.ones(3, 4, device=device, requires_grad=True))


@pytest.mark.parametrize("nhs", [(4, 4, 6), (1,), (8, 2, 3, 1, 4)])
def test_attention_norm_one_pass_equals_per_layer(nhs, device):
    """gatx_attention_norm_multi (round 6: every layer's alpha in one pass over edge_index') is
    bitwise the per-layer gatx_attention_norm launches accumulated in layer order
    (models/GATModel.py:189-234)."""
    import gatx
    from gatx import data as gd
    from gatx._lib import call, lib, ptr, stream
    from gatx.functional import _dst_row, attention_norm
    from gatx.graph import graph_cache
    b = gd.uniform_graph_batch(3, 700, 9000, 8, feature_seed=3)
    ei = torch.from_numpy(b.edge_index).to(device)
    gatx.clear_graph_cache()
    g = graph_cache.get(ei, b.num_nodes, True)
    E2 = g.num_edges
    gen = torch.Generator(device=device).manual_seed(9)
    alphas = [torch.rand(E2, nh, device=device, generator=gen) for nh in nhs]
    one = attention_norm(g.edge_index, alphas)
    out = torch.empty(1, dtype=torch.float32, device=device)
    ws = torch.empty(lib.gatx_attention_norm_workspace_bytes(), dtype=torch.uint8, device=device)
    scale = 1.0 / (E2 * len(alphas))
    for i, a in enumerate(alphas):
        call("gatx_attention_norm", ptr(a), E2, a.size(1), *_dst_row(g), ptr(g.rowptr), scale,
             int(i > 0), ptr(out), ptr(ws), stream())
    assert torch.equal(one.view(1), out)
