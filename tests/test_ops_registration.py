"""torch.library registration of the gatx ops (CPU: schemas, fake kernels, autograd formula
traced symbolically — no kernel runs). The GPU side (compiled model == eager goldens) is in
tests/test_gpu_compile.py."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gat-pytorch_amd")]

import torch  # noqa: E402
from torch.fx.experimental.proxy_tensor import make_fx  # noqa: E402

import gatx.layer  # noqa: E402,F401  (registers torch.ops.gatx.*)


def test_ops_registered():
    for name in ("layer_fwd", "layer_bwd", "attention_norm", "attention_norm_bwd"):
        assert hasattr(torch.ops.gatx, name), name
    sch = str(torch.ops.gatx.layer_fwd.default._schema)
    assert sch.startswith("gatx::layer_fwd(Tensor x, Tensor edge_index, Tensor W, Tensor? a")
    assert "-> (Tensor, Tensor, Tensor, Tensor[])" in sch


@pytest.mark.parametrize("concat,self_loops,F_in", [(True, True, 64), (False, True, 64),
                                                    (True, False, 64), (True, True, 50)])
def test_fake_layer_forward_backward(concat, self_loops, F_in):
    """Forward + backward of one layer traced with symbolic fake tensors: output shapes, the
    unbacked |edge_index'|, and a backward graph that calls gatx::layer_bwd."""
    NH, F, N, E = 4, 256, 300, 2000

    def f(x, ei, W, a):
        out, ei2, alpha, state = torch.ops.gatx.layer_fwd(x, ei, W, a, None, None, None, NH, F,
                                                          concat, self_loops, False, 0.0, True)
        loss = out.sum() + alpha.sum()
        gx, gW, ga = torch.autograd.grad(loss, (x, W, a))
        return out, ei2, alpha, gx, gW, ga

    x = torch.randn(N, F_in, requires_grad=True)
    ei = torch.randint(0, N, (2, E))
    W = torch.randn(NH * F, F_in, requires_grad=True)
    a = torch.randn(NH, NH * 2 * F, requires_grad=True)
    gm = make_fx(f, tracing_mode="symbolic")(x, ei, W, a)
    code = gm.code
    assert "gatx.layer_fwd" in code and "gatx.layer_bwd" in code
    outs = [n for n in gm.graph.nodes if n.op == "output"][0].args[0]
    out, ei2, alpha, gx, gW, ga = (n.meta["val"] for n in outs)
    assert tuple(out.shape) == (N, NH * F if concat else F)
    assert tuple(gx.shape) == (N, F_in) and tuple(gW.shape) == tuple(W.shape)
    assert tuple(ga.shape) == tuple(a.shape)
    assert alpha.shape[1] == NH and ei2.shape[0] == 2
    if self_loops:   # data-dependent |edge_index'|: an unbacked symbol shared by both outputs
        assert not isinstance(alpha.shape[0], int) and str(alpha.shape[0]) == str(ei2.shape[1])
        assert ei2.dtype == torch.int64
    else:
        assert int(alpha.shape[0]) == E


def test_fake_attention_norm():
    def f(ei, a1, a2):
        v = torch.ops.gatx.attention_norm(ei, [a1, a2])
        return torch.autograd.grad(v, (a1, a2))

    ei = torch.randint(0, 50, (2, 400))
    a1 = torch.rand(400, 4, requires_grad=True)
    a2 = torch.rand(400, 6, requires_grad=True)
    gm = make_fx(f, tracing_mode="symbolic")(ei, a1, a2)
    assert "gatx.attention_norm_bwd" in gm.code
