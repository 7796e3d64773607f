"""Autograd wiring of the fused GAT layer: forward = projection GEMM (+ per-node attention scores)
-> global max -> fused edge pass; backward = dst pass -> max() backward -> src pass -> two GEMMs
-> weight-gradient fix-ups. All device work is in libgatx.so (csrc/); this file only allocates
tensors from torch's caching allocator and launches on torch's current stream.

Reference: models/gat_layer.py:42-140 (forward); its autograd is restated in closed form in
SURVEY.md §8(a) a14 and oracle/gat_oracle.py:gat_layer_backward.
"""
from __future__ import annotations

import torch

from ._lib import ARGMAX_CAP, call, lib, ptr, stream
from .graph import Graph


class KernelTimer:
    """Optional HIP-event bracketing of the forward's launches (bench.py's live per-kernel
    timing). Events are recorded on torch's current stream — the stream every gatx launch uses."""

    def __init__(self):
        self.records = []   # (phase, info, start_event, end_event)

    def span(self, phase, info):
        timer = self

        class _Span:
            def __enter__(self):
                self.s = torch.cuda.Event(enable_timing=True)
                self.e = torch.cuda.Event(enable_timing=True)
                self.s.record()
                return self

            def __exit__(self, *exc):
                self.e.record()
                timer.records.append((phase, info, self.s, self.e))
                return False
        return _Span()

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for phase, info, s, e in self.records:
            out.setdefault(phase, []).append((info, s.elapsed_time(e)))
        return out


_timer: "KernelTimer | None" = None


def set_kernel_timer(t):
    global _timer
    _timer = t


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _span(phase, info):
    return _timer.span(phase, info) if _timer is not None else _Null()


def _round4(v: int) -> int:
    return (v + 3) // 4 * 4


def _require(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"gatx: {name} must be on the HIP device (no CPU path)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"gatx: {name} must be float32, got {t.dtype}")


class LayerShape:
    def __init__(self, num_heads: int, out_features: int, in_features: int, concat: bool,
                 const_attention: bool):
        self.NH, self.F, self.F_in = num_heads, out_features, in_features
        self.concat, self.const = bool(concat), bool(const_attention)
        self.Fp = _round4(out_features)
        self.Dp = self.NH * self.Fp
        self.H2 = 0 if self.const else 2 * self.NH
        self.K_aug = self.Dp + self.H2
        self.ldg = _round4(self.K_aug)
        self.out_cols = self.NH * self.F if self.concat else self.F


def project(x: torch.Tensor, W: torch.Tensor, a, sh: LayerShape):
    """Wh [N][Dp] and S [N][2NH] = x . W_aug^T in one MFMA GEMM (gat_layer.py:64 + :76-82)."""
    N = x.size(0)
    s = stream()
    waug_floats = lib.gatx_prepare_weights_floats(sh.NH, sh.F, sh.F_in, int(a is not None))
    W_aug = torch.empty(waug_floats, dtype=torch.float32, device=x.device)
    with _span("prepare_weights", (sh.NH, sh.F, sh.F_in)):
        call("gatx_prepare_weights", ptr(W), ptr(a), sh.NH, sh.F, sh.F_in, ptr(W_aug), s)
    Wh = torch.empty((N, sh.Dp), dtype=torch.float32, device=x.device)
    S = torch.empty((N, max(sh.H2, 1)), dtype=torch.float32, device=x.device)
    with _span("gemm", (N, sh.K_aug, sh.F_in, sh.NH, sh.F)):
        call("gatx_gemm_f32", N, sh.K_aug, sh.F_in, ptr(x), sh.F_in, 1, ptr(W_aug), 1, sh.F_in,
             ptr(Wh), sh.Dp, sh.Dp, ptr(S), max(sh.H2, 1), 0, s)
    return W_aug, Wh, S


def layer_forward(x, W, a, bias, graph: Graph, sh: LayerShape, p: float, seed: int):
    """Returns out, alpha (edge_index' order) and the saved state for the backward."""
    N = x.size(0)
    dev = x.device
    s = stream()
    W_aug, Wh, S = project(x, W, a, sh)
    M_ord = torch.zeros(1, dtype=torch.int32, device=dev)
    E2 = graph.num_edges
    if not sh.const:
        with _span("attention_max", (E2, sh.NH)):
            call("gatx_attention_max", ptr(graph.col), ptr(graph.rowidx), E2, ptr(S), sh.NH,
                 ptr(M_ord), s)
    out = torch.empty((N, sh.out_cols), dtype=torch.float32, device=dev)
    alpha = torch.empty((E2, sh.NH), dtype=torch.float32, device=dev)
    den = torch.empty((N, sh.NH), dtype=torch.float32, device=dev)
    argmax = torch.zeros(ARGMAX_CAP + 2, dtype=torch.int64, device=dev)
    with _span("edge_forward", (N, E2, sh.NH, sh.F, sh.concat)):
        call("gatx_edge_forward", ptr(Wh), ptr(S), ptr(M_ord), ptr(graph.rowptr),
             ptr(graph.col), ptr(graph.perm), N, sh.NH, sh.F, int(sh.concat), int(sh.const),
             ptr(bias), float(p), seed, ptr(out), ptr(alpha), ptr(den), ptr(argmax), s)
    saved = dict(W_aug=W_aug, Wh=Wh, S=S, M_ord=M_ord, den=den, argmax=argmax)
    return out, alpha, saved


def layer_backward(g_out, g_alpha, x, W, a, bias, graph: Graph, sh: LayerShape, p: float,
                   seed: int, saved, need_x: bool, need_W: bool, need_a: bool, need_bias: bool):
    N = x.size(0)
    dev = x.device
    s = stream()
    g_out = g_out.contiguous()
    E2 = graph.num_edges
    graph.ensure_transpose()
    G_aug = torch.empty((N, sh.ldg), dtype=torch.float32, device=dev)
    if not sh.const:
        g_raw = torch.empty((max(E2, 1), sh.NH), dtype=torch.float32, device=dev)
        n_part = lib.gatx_edge_backward_dst_partials(N)
        partials = torch.empty(n_part, dtype=torch.float32, device=dev)
        call("gatx_edge_backward_dst", ptr(saved["Wh"]), ptr(saved["S"]), ptr(saved["M_ord"]),
             ptr(saved["den"]), ptr(graph.rowptr), ptr(graph.col), ptr(graph.perm), N, sh.NH,
             sh.F, int(sh.concat), float(p), seed, ptr(g_out),
             ptr(g_alpha.contiguous()) if g_alpha is not None else None, ptr(g_raw), ptr(G_aug),
             sh.ldg, ptr(partials), s)
        g_corr = torch.zeros((N, sh.NH), dtype=torch.float32, device=dev)
        call("gatx_max_backward", ptr(partials), n_part, ptr(saved["argmax"]), ptr(saved["S"]),
             ptr(saved["M_ord"]), ptr(graph.col), ptr(graph.rowidx), E2, sh.NH, ptr(g_corr),
             ptr(G_aug), sh.ldg, sh.Dp, s)
    else:
        g_raw = g_corr = None
    call("gatx_edge_backward_src", ptr(saved["S"]), ptr(saved["M_ord"]), ptr(saved["den"]),
         ptr(graph.srowptr), ptr(graph.scol), ptr(graph.seid), ptr(graph.perm), N, sh.NH, sh.F,
         int(sh.concat), int(sh.const), float(p), seed, ptr(g_out), ptr(g_raw), ptr(g_corr),
         ptr(G_aug), sh.ldg, s)
    g_x = g_W = g_a = g_bias = None
    W_aug = saved["W_aug"]
    if need_x:
        g_x = torch.empty((N, sh.F_in), dtype=torch.float32, device=dev)
        call("gatx_gemm_f32", N, sh.F_in, sh.K_aug, ptr(G_aug), sh.ldg, 1, ptr(W_aug), sh.F_in, 1,
             ptr(g_x), sh.F_in, sh.F_in, None, 0, 0, s)
    if need_W or need_a:
        gW_aug = torch.empty((sh.K_aug, sh.F_in), dtype=torch.float32, device=dev)
        call("gatx_gemm_f32", sh.K_aug, sh.F_in, N, ptr(G_aug), 1, sh.ldg, ptr(x), sh.F_in, 1,
             ptr(gW_aug), sh.F_in, sh.F_in, None, 0, 0, s)
        g_W = torch.empty_like(W)
        g_a = torch.empty_like(a) if a is not None else None
        call("gatx_weight_grads", ptr(gW_aug), ptr(W), ptr(a), sh.NH, sh.F, sh.F_in, ptr(g_W),
             ptr(g_a), s)
    if need_bias and bias is not None:
        g_bias = torch.empty_like(bias)
        call("gatx_colsum", ptr(g_out), N, sh.out_cols, sh.out_cols, ptr(g_bias), s)
        if not sh.concat and bias.numel() != sh.out_cols:
            raise RuntimeError("bias with head-mean needs num_heads == 1")
    return g_x, (g_W if need_W else None), (g_a if need_a else None), g_bias


class GATLayerFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, a, bias, graph, sh, p, seed):
        out, alpha, saved = layer_forward(x, W, a, bias, graph, sh, p, seed)
        ctx.graph, ctx.sh, ctx.p, ctx.seed, ctx.saved = graph, sh, p, seed, saved
        ctx.save_for_backward(x, W, a, bias)
        return out, alpha

    @staticmethod
    def backward(ctx, g_out, g_alpha):
        x, W, a, bias = ctx.saved_tensors
        if g_out is None:
            g_out = torch.zeros((x.size(0), ctx.sh.out_cols), dtype=torch.float32,
                                device=x.device)
        nx, nW, na, nb = ctx.needs_input_grad[:4]
        g_x, g_W, g_a, g_b = layer_backward(g_out, g_alpha, x, W, a, bias, ctx.graph, ctx.sh,
                                            ctx.p, ctx.seed, ctx.saved, nx, nW, na, nb)
        return g_x, g_W, g_a, g_b, None, None, None, None


def gat_layer(x, edge_index, W, a, bias, num_heads, out_features, concat, add_self_loops,
              const_attention=False, dropout_p=0.0, seed=0, graph: Graph | None = None):
    """Functional form of GATLayer.forward: returns (out, edge_index', alpha)."""
    from .graph import graph_cache
    _require(x, "x")
    _require(W, "W")
    if a is not None:
        _require(a, "a")
    if bias is not None:
        _require(bias, "bias")
    if x.dim() != 2:
        raise RuntimeError(f"x must be (N, in_features), got {tuple(x.shape)}")
    x = x.contiguous()
    W = W.contiguous()
    a = a.contiguous() if a is not None else None
    sh = LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
    if W.shape != (num_heads * out_features, x.size(1)):
        raise RuntimeError(f"W.weight shape {tuple(W.shape)} does not match "
                           f"({num_heads * out_features}, {x.size(1)})")
    if graph is None:
        graph = graph_cache.get(edge_index, x.size(0), add_self_loops)
    if graph.num_edges == 0 and not const_attention:
        # attention_weights.max() of an empty tensor (models/gat_layer.py:85)
        raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
    if bias is not None and not concat and num_heads != 1:
        # output (N, F) += bias_param (NH*F,) cannot broadcast (models/gat_layer.py:134-135)
        raise RuntimeError(f"The size of tensor a ({out_features}) must match the size of tensor "
                           f"b ({num_heads * out_features}) at non-singleton dimension 1")
    out, alpha = GATLayerFunction.apply(x, W, a, bias, graph, sh, float(dropout_p), int(seed))
    return out, graph.edge_index, alpha
