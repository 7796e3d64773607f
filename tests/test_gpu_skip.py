"""GATModel's Linear skip on the gatx GEMMs (functional.SkipProjectionFunction) against fp64
torch: concat (x W^T) and head mean (mean_h x W_h^T as one product with the mean weight),
forward and both gradients. Model-level parity with the Linear skips is covered by the PATTERN
golden (tests/test_gpu_layer.py: every PATTERN layer has one)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("N,F_in,NH,F", [(952, 3, 4, 12), (952, 48, 4, 24), (952, 96, 4, 12),
                                          (952, 48, 1, 1), (3001, 200, 6, 37)])
def test_skip_projection_vs_fp64(N, F_in, NH, F, mean, device):
    from gatx.functional import SkipProjectionFunction
    g = torch.Generator(device=device).manual_seed(N + F_in)
    x = torch.randn(N, F_in, device=device, generator=g).requires_grad_(True)
    W = torch.randn(NH * F, F_in, device=device, generator=g).requires_grad_(True)
    out = SkipProjectionFunction.apply(x, W, NH, F, mean)
    go = torch.randn(out.shape, device=device, generator=g)
    (out * go).sum().backward()
    xd, Wd = x.detach().double().requires_grad_(True), W.detach().double().requires_grad_(True)
    ref = xd @ Wd.t()
    if mean:
        ref = ref.view(N, NH, F).mean(dim=1)
    (ref * go.double()).sum().backward()
    scale = lambda t: 1e-5 * max(1.0, t.abs().max().item())   # noqa: E731
    assert (out.double() - ref).abs().max().item() <= scale(ref)
    assert (x.grad.double() - xd.grad).abs().max().item() <= scale(xd.grad)
    assert (W.grad.double() - Wd.grad).abs().max().item() <= scale(Wd.grad)
