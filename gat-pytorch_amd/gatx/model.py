"""`GATModel` — the reference's layer stack (`models/GATModel.py:19-234`) without Lightning.

Builds `num_layers` gatx GATLayers exactly as `GATModel.__init__` does (`:64-116`: heads list
prefixed with 1, add_self_loops=True, bias=False, skip = Identity when widths match else a bias-free
Linear), and runs the same `forward` (`:120-151`) / `forward_and_return_attention` (`:153-187`)
wiring: input dropout -> layer -> skip (concat: add; mean: add head-mean of the skip) -> ELU except
after the last layer. `calc_attention_norm` restates `:189-234`. Submodule names
(`gat_layer_list.{i}.W.weight`, `.a.weight`, `skip_layer_list.{j}.weight`) match the reference's
state-dict keys, so its checkpoints load (see gatx.checkpoint.read_state_dict).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn.functional as F
from torch import nn

from .functional import side_alpha
from .graph import join_side
from .layer import GATLayer

# Linear skips of at least this many multiply-adds run on the gatx GEMM (x3: the PPI-scale
# products, e.g. the notebook variant's 44900 x 1024 x 1024 skip, where hipBLASLt's fp32 path is
# ~1.6x slower); smaller ones stay nn.Linear: at PATTERN's 952 x 96 x 48 a vendor launch takes
# ~5 us against 6-14 us for the tiled / small-K gatx kernels (profiles/r02d_small)
SKIP_GEMM_MIN_MACS = 1 << 26


def _dropout_fuse_enabled() -> bool:
    """tuning dropout_fuse=0 applies every input dropout with the standalone gatx kernel instead
    of the producing layer's epilogue (A/B tests)."""
    from . import tuning
    return tuning.get("dropout_fuse") != 0


def _skip_fold_enabled() -> bool:
    """tuning skip_fold=0 turns the folded skip projection off (A/B tests and measurements)."""
    from . import tuning
    return tuning.get("skip_fold") != 0


class GATModel(nn.Module):
    def __init__(self, num_classes: int, num_input_node_features: int, num_layers: int,
                 num_heads_per_layer: List[int], heads_concat_per_layer: List[bool],
                 head_output_features_per_layer: List[int], add_skip_connection: List[bool],
                 dropout: float, const_attention: bool = False, **kwargs):
        super().__init__()
        self.num_layers = num_layers
        self.dropout = dropout
        self.num_classes = num_classes
        self.add_skip_connection = add_skip_connection
        self.num_heads_per_layer = [1] + list(num_heads_per_layer)
        self.head_output_features_per_layer = head_output_features_per_layer
        self.heads_concat_per_layer = heads_concat_per_layer
        self.const_attention = const_attention
        self.lr = kwargs.get("learning_rate", 0.005)
        self.l2_reg = kwargs.get("l2_reg", 0.0)
        gat_layers, skip_layers = [], []
        for i in range(num_layers):
            fin = self.num_heads_per_layer[i] * head_output_features_per_layer[i]
            gat_layers.append(GATLayer(
                in_features=fin, out_features=head_output_features_per_layer[i + 1],
                num_heads=self.num_heads_per_layer[i + 1], concat=heads_concat_per_layer[i],
                dropout=dropout, bias=False, add_self_loops=True,
                const_attention=const_attention))
            if add_skip_connection[i]:
                skip_out = self.num_heads_per_layer[i + 1] * head_output_features_per_layer[i + 1]
                skip_layers.append(nn.Identity() if fin == skip_out
                                   else nn.Linear(fin, skip_out, bias=False))
        self.gat_layer_list = nn.ModuleList(gat_layers)
        self.skip_layer_list = nn.ModuleList(skip_layers)
        # True: skip / ELU / dropout fused into the layers (gatx's wiring). False: the
        # reference's own forward (`models/GATModel.py:120-151`) op for op around gatx GATLayers —
        # exactly what the INTEGRATION.md §1 drop-in (swap the import) runs; bench.py
        # --wiring reference times it
        self.fuse_wiring = True

    def _resid(self, i, skip_count, layer_input):
        """Skip connection of layer i (`models/GATModel.py:135-145`) in the layer's output shape,
        to be added inside the layer's fused epilogue. A Linear skip runs on the gatx GEMMs
        (functional.SkipProjectionFunction; its head mean folded into the weight), except while
        torch.compile traces (plain torch ops, which the compiler handles itself)."""
        skip = self.skip_layer_list[skip_count]
        nh, f = self.num_heads_per_layer[i + 1], self.head_output_features_per_layer[i + 1]
        mean = not self.heads_concat_per_layer[i]
        if (isinstance(skip, nn.Linear) and not torch.compiler.is_compiling()
                and layer_input.size(0) * skip.weight.numel() >= SKIP_GEMM_MIN_MACS):
            from .functional import SkipProjectionFunction
            return SkipProjectionFunction.apply(layer_input, skip.weight, nh, f, mean)
        skip_output = skip(layer_input)
        if not mean:
            return skip_output
        return skip_output.view(-1, nh, f).mean(dim=1)

    def _fuse_next_dropout(self, i) -> bool:
        """Layer i applies layer i+1's input dropout in its epilogue: layer i+1 has no skip (the
        skip reads the undropped input) and layer i's output comes from the edge pass."""
        from .functional import fuses_output_dropout
        if i + 1 >= len(self.gat_layer_list) or self.add_skip_connection[i + 1]:
            return False
        lay = self.gat_layer_list[i]
        return _dropout_fuse_enabled() and fuses_output_dropout(
            lay.num_heads, lay.out_features, lay.in_features, lay.concat, lay.const_attention)

    def _run_reference_wiring(self, x, edge_index, with_attention):
        """`models/GATModel.py:153-187` with the gatx layer: dropout, layer, skip module (+ head
        mean), add, ELU as separate torch ops."""
        attention_weights_list = []
        skip_count = 0
        L = len(self.gat_layer_list)
        for i in range(L):
            layer_input = x
            x = F.dropout(x, p=self.dropout, training=self.training)
            out = self.gat_layer_list[i](x, edge_index, return_attention_weights=with_attention)
            if with_attention:
                x, (edge_index, att) = out
                attention_weights_list.append(att)
            else:
                x = out
            if self.add_skip_connection[i]:
                skip_output = self.skip_layer_list[skip_count](layer_input)
                skip_count += 1
                if self.heads_concat_per_layer[i]:
                    x = x + skip_output
                else:
                    skip_output = skip_output.view(-1, self.num_heads_per_layer[i + 1],
                                                   self.head_output_features_per_layer[i + 1])
                    x = x + skip_output.mean(dim=1)
            if i != L - 1:
                x = F.elu(x)
        return x, edge_index, attention_weights_list

    def _run(self, x, edge_index, with_attention):
        if not self.fuse_wiring:
            return self._run_reference_wiring(x, edge_index, with_attention)
        attention_weights_list = []
        skip_count = 0
        L = len(self.gat_layer_list)
        # input dropout (models/GATModel.py:130) on gatx's counter-based mask: one device seed per
        # layer input drawn up front (the same draws whichever way each dropout is applied),
        # applied by the producing layer's epilogue where it can be, else by gatx_dropout
        gx_drop = (self.training and self.dropout > 0 and x.is_cuda
                   and not torch.compiler.is_compiling())
        seeds = ([torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=x.device)
                  for _ in range(L)] if gx_drop else None)
        pre_dropped = False
        for i in range(L):
            layer_input = x
            if gx_drop:
                if not pre_dropped:
                    from .functional import input_dropout
                    x = input_dropout(x, self.dropout, seeds[i])
            else:
                x = F.dropout(x, p=self.dropout, training=self.training)
            fuse_next = gx_drop and self._fuse_next_dropout(i)
            resid = skip_w = None
            if self.add_skip_connection[i]:
                skip = self.skip_layer_list[skip_count]
                if (isinstance(skip, nn.Linear) and (self.dropout == 0 or not self.training)
                        and not torch.compiler.is_compiling() and _skip_fold_enabled()):
                    # the skip reads the layer's own input (no input dropout in effect): its
                    # projection is folded into the layer's projection GEMM (one launch)
                    skip_w = skip.weight
                else:
                    resid = self._resid(i, skip_count, layer_input)
                skip_count += 1
            # layer -> (+ skip) -> ELU except after the last layer, fused in the layer epilogue
            extra = {"skip_weight": skip_w} if skip_w is not None else {}
            if fuse_next:
                extra["out_dropout"] = (self.dropout, seeds[i + 1])
            pre_dropped = fuse_next
            # all but the last layer: the alpha pass runs on the side stream under the next
            # layer's projection GEMM (functional.side_alpha; joined there and below)
            with side_alpha(i != L - 1 and x.is_cuda and not torch.compiler.is_compiling()):
                out = self.gat_layer_list[i](x, edge_index,
                                             return_attention_weights=with_attention,
                                             resid=resid, elu=(i != L - 1), **extra)
            if with_attention:
                x, (edge_index, att) = out
                attention_weights_list.append(att)
            else:
                x = out
        if x.is_cuda:
            join_side(x.device)
        return x, edge_index, attention_weights_list

    @staticmethod
    def _unpack(x, edge_index):
        # the reference takes a PyG-style batch (`data.x`, `data.edge_index`); tensors also work
        if edge_index is None:
            if not (hasattr(x, "x") and hasattr(x, "edge_index")):
                raise TypeError("GATModel: pass (x, edge_index) or an object with .x and "
                                ".edge_index")
            return x.x, x.edge_index
        return x, edge_index

    def forward(self, x, edge_index=None):
        """`models/GATModel.py:120-151` (`forward(data)`, or `forward(x, edge_index)`): dropout
        -> layer -> skip -> ELU, per layer. In training with dropout the masks are gatx's
        counter-based ones (torch's RNG stream cannot be matched bit for bit); the next layer's
        dropout rides on the layer's epilogue."""
        return self._run(*self._unpack(x, edge_index), False)[0]

    def forward_and_return_attention(self, x, edge_index=None, return_attention_weights=True):
        """`models/GATModel.py:153-187` (`(data)` or `(x, edge_index)`): as forward, also
        returning edge_index' and the alphas."""
        return self._run(*self._unpack(x, edge_index), True)

    @staticmethod
    def calc_attention_norm(edge_index, attention_list):
        """mean over layers of ||alpha * in_degree[dst] - 1||_1 / E (`models/GATModel.py:189-234`),
        fused on the device (gatx_attention_norm; degrees from the cached CSR of edge_index')."""
        if torch.compiler.is_compiling():
            return torch.ops.gatx.attention_norm(edge_index, list(attention_list))
        from .functional import attention_norm
        return attention_norm(edge_index, attention_list)

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr, weight_decay=self.l2_reg)
