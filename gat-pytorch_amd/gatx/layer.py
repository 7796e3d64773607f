"""`GATLayer` — drop-in for the reference's `models/gat_layer.py:GATLayer`, running on libgatx.

Same constructor signature, attributes, submodules and state-dict keys as the reference
(`models/gat_layer.py:13-40`): `W` (nn.Linear, no bias), `a` (nn.Linear NH*2F -> NH, absent when
const_attention), `bias_param` (when bias), `dropout_layer` (when dropout > 0), and the side effect
`self.normalised_attention_coeffs = alpha` of every forward (`:110`). So it plugs into GATModel
(`models/GATModel.py:69-79`), PPI_GAT / PlanetoidGAT / PatternGAT and their checkpoints unchanged.

forward(x, edge_index, return_attention_weights=False) -> out, or (out, (edge_index', alpha)),
exactly as `:42-140`. The computation is the reference's (including its quirks: the cross-head
`a` mixing, one global max subtracted before LeakyReLU(0.01), the 1e-8 softmax epsilon with no
per-segment max, isolated trailing nodes getting no self-loop), but fused into HIP kernels:
no per-edge (E, NH, F) tensor is ever built. There is deliberately no CPU path.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops  # noqa: F401  (registers torch.ops.gatx.*)
from .functional import LazyAlpha, gat_layer_lazy


class GATLayer(nn.Module):
    # Opt-in (default off, as the reference writes alpha in every forward, `:106-110`): with
    # lazy_alpha an inference forward (autograd off, no return_attention_weights) keeps the
    # softmax state and runs the alpha pass when normalised_attention_coeffs is first read
    # (functional.LazyAlpha: same kernel, same inputs, bitwise the same values).
    lazy_alpha = False

    def __init__(self, in_features, out_features, num_heads, concat, dropout=0,
                 add_self_loops=False, bias=False, const_attention=False):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.num_heads = num_heads
        self.concat = concat
        self.dropout = dropout
        self.add_self_loops = add_self_loops
        self.bias = bias
        self.const_attention = const_attention
        self.device = "cuda" if torch.cuda.is_available() else "cpu"

        self.W = nn.Linear(in_features=self.in_features,
                           out_features=self.num_heads * self.out_features, bias=False)
        if not const_attention:
            self.a = nn.Linear(in_features=self.num_heads * (2 * self.out_features),
                               out_features=self.num_heads, bias=False)
        if self.dropout > 0:
            self.dropout_layer = nn.Dropout(p=self.dropout)
        if self.bias:
            self.bias_param = nn.Parameter(torch.Tensor(self.num_heads * self.out_features))
        self.normalised_attention_coeffs = None
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.W.weight)
        if not self.const_attention:
            nn.init.xavier_uniform_(self.a.weight)
        if self.bias:
            nn.init.zeros_(self.bias_param)

    def _dropout_seed(self, device):
        # one 64-bit draw from torch's generator on the layer's device per forward (the
        # reference's nn.Dropout draws there too): follows torch.cuda.manual_seed, no host sync,
        # and a captured hipGraph draws a fresh seed on every replay
        return torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=device)

    @property
    def normalised_attention_coeffs(self):
        """alpha of the last forward (`models/gat_layer.py:110`), (E', NH) in edge_index' order.
        Kept at its allocation bound until read: the exact E' lives on the device, so the slice
        (one host read of E') happens here, not in forward. After an inference forward (autograd
        off, no return_attention_weights) of a layer with `lazy_alpha` set, the alpha pass itself
        runs on this first read (functional.LazyAlpha: same kernel, same inputs, same values)."""
        att = self.__dict__.get("_attention")
        if att is None or isinstance(att, torch.Tensor):
            return att
        graph, alpha = att
        if isinstance(alpha, LazyAlpha):   # an inference forward's alpha, computed on first read
            alpha = alpha.materialize()
        view = alpha[:graph.num_edges]
        self.__dict__["_attention"] = view
        return view

    @normalised_attention_coeffs.setter
    def normalised_attention_coeffs(self, value):
        self.__dict__["_attention"] = value

    def forward(self, x, edge_index, return_attention_weights=False, *, graph=None, resid=None,
                elu=False, skip_weight=None, out_dropout=None):
        """Reference signature (`models/gat_layer.py:42`); keyword-only extras: `graph` (a
        prebuilt gatx.Graph), `resid` / `elu` (GATModel's skip-add + ELU fused into the
        epilogue: returns elu?(out + resid)), `skip_weight` (GATModel's Linear skip weight,
        folded into this layer's projection GEMM: resid = x W_skip^T, or its head mean),
        `out_dropout` ((p, device seed): the next layer's input dropout applied by this layer's
        epilogue, gatx.functional.fuses_output_dropout). Without
        return_attention_weights nothing waits for the device (|edge_index'| is only known
        there)."""
        p = float(self.dropout) if (self.dropout > 0 and self.training) else 0.0
        if torch.compiler.is_compiling():
            # traced by torch.compile: the registered op (gatx/ops.py), opaque to the compiler
            if graph is not None or skip_weight is not None or out_dropout is not None:
                raise RuntimeError("gatx: graph= / skip_weight= / out_dropout= are not supported "
                                   "under torch.compile")
            seed_t = self._dropout_seed(x.device) if p > 0 else None
            out, ei2, alpha, _ = torch.ops.gatx.layer_fwd(
                x, edge_index, self.W.weight, None if self.const_attention else self.a.weight,
                self.bias_param if self.bias else None, resid, seed_t, self.num_heads,
                self.out_features, self.concat, self.add_self_loops, self.const_attention, p,
                elu)
            self.__dict__["_attention"] = alpha
            return (out, (ei2, alpha)) if return_attention_weights else out
        seed = self._dropout_seed(x.device) if p > 0 else 0
        defer = self.lazy_alpha and not return_attention_weights
        out, g, alpha = gat_layer_lazy(
            x, edge_index, self.W.weight, None if self.const_attention else self.a.weight,
            self.bias_param if self.bias else None, self.num_heads, self.out_features,
            self.concat, self.add_self_loops, self.const_attention, p, seed, graph=graph,
            resid=resid, elu=elu, skip_weight=skip_weight, out_dropout=out_dropout,
            defer_alpha=defer)
        self.normalised_attention_coeffs = (g, alpha)
        if return_attention_weights:
            return out, (g.edge_index, self.normalised_attention_coeffs)
        return out

    def extra_repr(self) -> str:
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"num_heads={self.num_heads}, concat={self.concat}, dropout={self.dropout}, "
                f"add_self_loops={self.add_self_loops}, bias={self.bias}, "
                f"const_attention={self.const_attention}")
