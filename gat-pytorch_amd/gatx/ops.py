"""torch.library registration of the gatx entry points: `torch.ops.gatx.*`.

The plugin point of the reference is the `nn.Module` (`models/gat_layer.py:6`, selected in
`models/GATModel.py:69-79`); the C-ABI (include/gatx.h) sits underneath it. These ops wrap the same
C-ABI calls as opaque operators with fake (meta) kernels and registered autograd, so that a model
built from gatx.GATLayer compiles under `torch.compile(fullgraph=True)` without graph breaks
(GATLayer.forward dispatches here while torch.compile traces; eager calls keep the sync-free
autograd.Function path of gatx.functional, which runs the same kernels):

  gatx::layer_fwd(x, edge_index, W, a?, bias?, resid?, seed?, num_heads, out_features, concat,
                  add_self_loops, const_attention, p, elu)
      -> (out, edge_index', alpha, state[])            models/gat_layer.py:42-140
  gatx::layer_bwd(g_out, g_alpha?, x, edge_index, W, a?, bias?, seed?, out?, state[], ...,
                  need_x, need_W, need_a, need_bias, need_resid, resid_is_x)
      -> [g_x, g_W, g_a, g_bias, g_resid]              autograd of the above
  gatx::attention_norm(edge_index', alphas[]) -> ()    models/GATModel.py:189-234
  gatx::attention_norm_bwd(edge_index', alphas[], g) -> [g_alpha...]

|edge_index'| is data dependent (the self-loop rewrite drops existing loops, `models/utils.py:
61-65`), so the fake kernel gives edge_index' / alpha an unbacked size. `state` carries the
forward's saved device tensors (W_aug, M_ord, den, argmax, S, Wh, Z, x_rows; empty = absent) to
the backward op. The layer's CSR is not an op argument: both ops take it from the graph cache
(gatx.graph), keyed on edge_index, exactly as the eager path does.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import functional as fn
from ._lib import ARGMAX_CAP, lib

_STATE = ("W_aug", "M_ord", "den", "argmax", "S", "Wh", "Z", "x_rows")


def _empty(dev):
    return torch.empty(0, dtype=torch.float32, device=dev)


def _state_shapes(sh: "fn.LayerShape", N, has_a: bool):
    """(shape, dtype) of each state tensor, in _STATE order (None: absent)."""
    waug = lib.gatx_prepare_weights_floats(sh.NH, sh.F, sh.F_in, int(has_a))
    f32, i32, i64 = torch.float32, torch.int32, torch.int64
    reassoc = fn.use_reassociation(sh)
    Fin_p = fn._round4(sh.F_in)
    return [((waug,), f32), ((1,), i32), ((N, sh.NH), f32), ((ARGMAX_CAP + 2,), i64),
            ((N, max(sh.H2, 1)), f32),
            None if reassoc else ((N, sh.Dp), f32),
            ((N, sh.NH * Fin_p), f32) if reassoc else None,
            ((N, Fin_p), f32) if (reassoc and Fin_p != sh.F_in) else None]


@torch.library.custom_op("gatx::layer_fwd", mutates_args=(), device_types="cuda")
def layer_fwd(x: Tensor, edge_index: Tensor, W: Tensor, a: Optional[Tensor],
              bias: Optional[Tensor], resid: Optional[Tensor], seed: Optional[Tensor],
              num_heads: int, out_features: int, concat: bool, add_self_loops: bool,
              const_attention: bool, p: float, elu: bool
              ) -> Tuple[Tensor, Tensor, Tensor, List[Tensor]]:
    x, W, a, resid, sh, graph = fn.prepare_layer(x, edge_index, W, a, bias, num_heads,
                                                 out_features, concat, add_self_loops,
                                                 const_attention, None, resid)
    out, alpha, saved = fn.layer_forward(x, W, a, bias, graph, sh, float(p), seed, resid, elu)
    E2 = graph.num_edges
    # edge_index' may not alias an input of the op (without the rewrite the reference returns its
    # input; a later layer is handed the previous layer's edge_index' itself): then a copy, which
    # the graph cache learns as another key of the same graph (the next layer / the attention
    # norm find the CSR instead of rebuilding it)
    from .graph import graph_cache
    ei2 = graph.edge_index
    if ei2.data_ptr() == edge_index.data_ptr() or not add_self_loops:
        ei2 = ei2.clone()
        graph_cache.alias(ei2, graph)
    dev = x.device
    xr = saved.get("x_rows")
    state = [saved["W_aug"], saved["M_ord"], saved["den"], saved["argmax"], saved["S"],
             saved["Wh"] if saved["Wh"] is not None else _empty(dev),
             saved["Z"] if saved.get("reassoc") else _empty(dev),
             xr if (xr is not None and xr is not x) else _empty(dev)]
    return out, ei2, alpha[:E2], state


@layer_fwd.register_fake
def _layer_fwd_fake(x, edge_index, W, a, bias, resid, seed, num_heads, out_features, concat,
                    add_self_loops, const_attention, p, elu):
    sh = fn.LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
    N = x.size(0)
    if add_self_loops:
        E2 = torch.library.get_ctx().new_dynamic_size()
        ei2 = edge_index.new_empty((2, E2), dtype=torch.int64)
    else:
        E2 = edge_index.size(1)
        ei2 = edge_index.new_empty((2, E2))
    out = x.new_empty((N, sh.out_cols))
    alpha = x.new_empty((E2, num_heads))
    state = [x.new_empty((0,)) if s is None else x.new_empty(s[0], dtype=s[1])
             for s in _state_shapes(sh, N, a is not None)]
    return out, ei2, alpha, state


def _saved_from_state(state, x):
    d = dict(zip(_STATE, state))
    saved = {k: d[k] for k in ("W_aug", "M_ord", "den", "argmax", "S")}
    saved["Wh"] = d["Wh"] if d["Wh"].numel() else None
    saved["reassoc"] = d["Z"].numel() > 0
    if saved["reassoc"]:
        saved["Z"] = d["Z"]
        saved["x_rows"] = d["x_rows"] if d["x_rows"].numel() else x
    return saved


@torch.library.custom_op("gatx::layer_bwd", mutates_args=(), device_types="cuda")
def layer_bwd(g_out: Tensor, g_alpha: Optional[Tensor], x: Tensor, edge_index: Tensor,
              W: Tensor, a: Optional[Tensor], bias: Optional[Tensor], seed: Optional[Tensor],
              out: Optional[Tensor], state: List[Tensor], num_heads: int, out_features: int,
              concat: bool, add_self_loops: bool, const_attention: bool, p: float, elu: bool,
              need_x: bool, need_W: bool, need_a: bool, need_bias: bool, need_resid: bool,
              resid_is_x: bool) -> List[Tensor]:
    from .graph import graph_cache
    x = x.contiguous()
    W = W.contiguous()
    a = a.contiguous() if a is not None else None
    sh = fn.LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
    sh.cache_weights = False
    graph = graph_cache.get(edge_index, x.size(0), add_self_loops)
    saved = _saved_from_state(state, x)
    g_x, g_W, g_a, g_b, g_r = fn.layer_backward(
        g_out, g_alpha, x, W, a, bias, graph, sh, float(p), seed, saved, need_x, need_W,
        need_a, need_bias, out=out, elu=elu, need_resid=need_resid, resid_is_x=resid_is_x)
    dev = x.device
    return [t if t is not None else _empty(dev) for t in (g_x, g_W, g_a, g_b, g_r)]


@layer_bwd.register_fake
def _layer_bwd_fake(g_out, g_alpha, x, edge_index, W, a, bias, seed, out, state, num_heads,
                    out_features, concat, add_self_loops, const_attention, p, elu, need_x,
                    need_W, need_a, need_bias, need_resid, resid_is_x):
    sh = fn.LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
    e = x.new_empty((0,))
    fold = resid_is_x and need_x and need_resid
    return [x.new_empty(x.shape) if need_x else e,
            W.new_empty(W.shape) if need_W else e,
            a.new_empty(a.shape) if (need_a and a is not None) else e,
            bias.new_empty(bias.shape) if (need_bias and bias is not None) else e,
            x.new_empty((x.size(0), sh.out_cols)) if (need_resid and not fold) else e]


def _layer_setup(ctx, inputs, output):
    (x, edge_index, W, a, bias, resid, seed, num_heads, out_features, concat, add_self_loops,
     const_attention, p, elu) = inputs
    out, _, _, state = output
    ctx.save_for_backward(x, edge_index, W, a, bias, seed, out if elu else None, *state)
    ctx.args = (num_heads, out_features, concat, add_self_loops, const_attention, p, elu)
    ctx.has_resid = resid is not None
    ctx.resid_is_x = resid is not None and resid is x


def _layer_backward(ctx, g_out, g_ei2, g_alpha, g_state):
    x, edge_index, W, a, bias, seed, out, *state = ctx.saved_tensors
    num_heads, out_features, concat, add_self_loops, const_attention, p, elu = ctx.args
    nx, _, nW, na, nb, nr = ctx.needs_input_grad[:6]
    if g_out is None:
        sh = fn.LayerShape(num_heads, out_features, x.size(1), concat, const_attention)
        g_out = x.new_zeros((x.size(0), sh.out_cols))
    need_resid = bool(ctx.has_resid and nr)
    g = torch.ops.gatx.layer_bwd(
        g_out.contiguous(), g_alpha, x, edge_index, W, a, bias, seed, out, state, num_heads,
        out_features, concat, add_self_loops, const_attention, p, elu, bool(nx), bool(nW),
        bool(na and a is not None), bool(nb and bias is not None), need_resid,
        bool(ctx.resid_is_x))
    g_x, g_W, g_a, g_b, g_r = g
    fold = ctx.resid_is_x and nx and need_resid
    return (g_x if nx else None, None, g_W if nW else None,
            g_a if (na and a is not None) else None, g_b if (nb and bias is not None) else None,
            g_r if (need_resid and not fold) else None,
            None, None, None, None, None, None, None, None)


layer_fwd.register_autograd(_layer_backward, setup_context=_layer_setup)


@torch.library.custom_op("gatx::attention_norm", mutates_args=(), device_types="cuda")
def attention_norm(edge_index: Tensor, alphas: List[Tensor]) -> Tensor:
    from .graph import graph_cache
    graph = graph_cache.for_edges(edge_index)
    return fn.AttentionNormFunction.forward(_Ctx(), graph, *alphas).clone()


@attention_norm.register_fake
def _attention_norm_fake(edge_index, alphas):
    return alphas[0].new_empty(())


@torch.library.custom_op("gatx::attention_norm_bwd", mutates_args=(), device_types="cuda")
def attention_norm_bwd(edge_index: Tensor, alphas: List[Tensor], g: Tensor) -> List[Tensor]:
    from .graph import graph_cache
    graph = graph_cache.for_edges(edge_index)
    ctx = _Ctx()
    ctx.graph = graph
    ctx.scale = 1.0 / (graph.num_edges * len(alphas)) if graph.num_edges else float("nan")
    ctx.saved_tensors = tuple(a.contiguous() for a in alphas)
    return list(fn.AttentionNormFunction.backward(ctx, g)[1:])


@attention_norm_bwd.register_fake
def _attention_norm_bwd_fake(edge_index, alphas, g):
    return [a.new_empty(a.shape) for a in alphas]


class _Ctx:
    """Stand-in for an autograd ctx when the ops call AttentionNormFunction's kernels directly."""

    def save_for_backward(self, *t):
        self.saved_tensors = t


def _norm_setup(ctx, inputs, output):
    edge_index, alphas = inputs
    ctx.save_for_backward(edge_index, *alphas)


def _norm_backward(ctx, g):
    edge_index, *alphas = ctx.saved_tensors
    return None, torch.ops.gatx.attention_norm_bwd(edge_index, alphas, g)


attention_norm.register_autograd(_norm_backward, setup_context=_norm_setup)
