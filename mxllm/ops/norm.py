"""RMSNorm (and residual-add + RMSNorm) with HIP forward/backward kernels.

SURVEY §2.4 K5.  On GPU both directions run ``csrc/kernels/rmsnorm.hip``;
the residual add of a transformer sub-block is fused into the norm that follows
it (forward) and the residual-gradient add into the norm's backward, which
removes a full read+write of the [T, H] residual stream per sub-block.
"""
from __future__ import annotations

import torch

from . import reference as ref
from ..parallel.grad_ready import accum_grad
from ._ext import native, rows_view, use_native

# ``out_pad`` / ``grad_pad``: the normalised output (forward) or the input
# gradient (backward) is written as the left [T, H] part of a [T, H + pad]
# buffer, so a LoRA projection consuming it can append its rank columns in
# place and run ONE augmented GEMM (mxllm/ops/linear.py).


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, out_pad):
        y, rstd, _ = native().rmsnorm_fwd(x, None, w, eps, out_pad)
        ctx.save_for_backward(x, w, rstd)
        ctx.wp = w if w.is_leaf else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx, dw = native().rmsnorm_bwd(dy.contiguous(), x, w, rstd, None, ctx.needs_input_grad[1])
        return dx, _wgrad(ctx, dw, w, 1), None, None


def _wgrad(ctx, dw, w, idx: int):
    """dγ (fp32 from the kernel; ``idx``: w's input position): added straight into
    an fp32 gradient target when the owner keeps one (no bf16 rounding), else
    handed to autograd as w.dtype."""
    if dw is None or not ctx.needs_input_grad[idx]:
        return None
    if accum_grad(ctx.wp, dw):
        return None
    return dw.to(w.dtype)


class _AddRMSNormFn(torch.autograd.Function):
    """(x, res, w) -> (y = rmsnorm(x + res) * w, h = x + res)."""

    @staticmethod
    def forward(ctx, x, res, w, eps, out_pad, grad_pad):
        y, rstd, h = native().rmsnorm_fwd(x, res, w, eps, out_pad)
        ctx.save_for_backward(h, w, rstd)
        ctx.wp = w if w.is_leaf else None
        ctx.grad_pad = grad_pad
        return y, h

    @staticmethod
    def backward(ctx, dy, dh):
        h, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        dres = rows_view(dh) if dh is not None else None
        dx, dw = native().rmsnorm_bwd(dy.contiguous(), h, w, rstd, dres, ctx.needs_input_grad[2], ctx.grad_pad)
        return dx, dx, _wgrad(ctx, dw, w, 2), None, None, None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5, out_pad: int = 0) -> torch.Tensor:
    if use_native(x):
        if out_pad and x.dim() != 2:
            out_pad = 0
        return _RMSNormFn.apply(x.contiguous(), w, eps, out_pad)
    return ref.rms_norm(x, w, eps)


def add_rms_norm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float = 1e-5, out_pad: int = 0,
                 grad_pad: int = 0):
    """Returns (normed, new_residual) where new_residual = x + res.
    ``out_pad``: pad columns behind the normed rows (consumer: a LoRA GEMM);
    ``grad_pad``: the same for the gradient of ``x`` (producer of x: a LoRA GEMM)."""
    if use_native(x):
        if x.dim() != 2:
            out_pad = grad_pad = 0
        return _AddRMSNormFn.apply(x.contiguous(), res.contiguous(), w, eps, out_pad, grad_pad)
    h = x + res
    return ref.rms_norm(h, w, eps), h
