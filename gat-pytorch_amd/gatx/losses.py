"""The task modules' loss on the device, fused (csrc/loss.hip): BCEWithLogitsLoss with mean
reduction and an optional scalar pos_weight — PPI_GAT's `nn.BCEWithLogitsLoss()`
(`models/ppi_gat.py:11,19`) and PatternGAT's `nn.BCEWithLogitsLoss(pos_weight=1/0.1765)`
(`models/pattern_gat.py:11-15`). One launch computes the loss and its gradient; the backward is
one scaling launch (torch: ~19 launches for forward + backward)."""
from __future__ import annotations

import torch

from ._lib import call, lib, ptr, stream
from .functional import _span


class BCEWithLogitsFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, pos_weight: float):
        if not (x.is_cuda and y.is_cuda):
            raise RuntimeError("gatx: bce_with_logits needs HIP tensors (no CPU path)")
        if x.dtype != torch.float32 or y.dtype != torch.float32:
            raise RuntimeError("gatx: bce_with_logits needs float32 input and target")
        if y.requires_grad:
            # the fused kernel writes d loss / d input only; torch would also differentiate the
            # target (-x / n + (pos_weight - 1) softplus(-x) / n): refuse rather than drop it
            raise RuntimeError("gatx: bce_with_logits does not differentiate the target; pass "
                               "target.detach() (the task modules' targets are labels)")
        if x.shape != y.shape:
            raise ValueError(f"Target size ({tuple(y.shape)}) must be the same as input size "
                             f"({tuple(x.shape)})")
        x = x.contiguous()
        y = y.contiguous()
        n = x.numel()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        grad = torch.empty_like(x)
        ws = None
        if n > (1 << 16):
            ws = torch.empty(lib.gatx_bce_logits_workspace_bytes(), dtype=torch.uint8,
                             device=x.device)
        with _span("bce", (n,)):
            call("gatx_bce_logits", ptr(x), ptr(y), n, float(pos_weight), ptr(loss), ptr(grad),
                 ptr(ws), stream())
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        out = torch.empty_like(grad)
        with _span("bce_bwd", (grad.numel(),)):
            call("gatx_scale_by_scalar", ptr(g.to(torch.float32).contiguous()), ptr(grad),
                 grad.numel(), ptr(out), stream())
        return out, None, None


def bce_with_logits(input: torch.Tensor, target: torch.Tensor, pos_weight=None) -> torch.Tensor:
    """torch.nn.functional.binary_cross_entropy_with_logits(input, target, pos_weight=pos_weight)
    (mean reduction) on the device; pos_weight: None, a float or a one-element tensor (read once
    on the host — build the loss outside a captured step's first run)."""
    if pos_weight is None:
        pw = 1.0
    elif isinstance(pos_weight, torch.Tensor):
        if pos_weight.numel() != 1:
            raise ValueError("gatx: bce_with_logits supports a scalar pos_weight")
        pw = float(pos_weight.item())
    else:
        pw = float(pos_weight)
    return BCEWithLogitsFunction.apply(input, target, pw)


class BCEWithLogitsLoss(torch.nn.Module):
    """nn.BCEWithLogitsLoss(pos_weight=...) (mean) on gatx's fused kernels. pos_weight is read
    once, at construction."""

    def __init__(self, pos_weight=None):
        super().__init__()
        if isinstance(pos_weight, torch.Tensor):
            if pos_weight.numel() != 1:
                raise ValueError("gatx: BCEWithLogitsLoss supports a scalar pos_weight")
            pos_weight = float(pos_weight.item())
        self.pw = 1.0 if pos_weight is None else float(pos_weight)

    def forward(self, input, target):
        return BCEWithLogitsFunction.apply(input, target, self.pw)
