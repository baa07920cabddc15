"""Fused AdamW over flat parameter buffers.

mxllm keeps every trainable parameter as a view into ONE flat fp32 master
buffer (and, for full fine-tuning, one flat bf16 compute buffer); gradients
land in one flat buffer too.  The optimizer step is therefore a single
vectorised HIP kernel launch per weight-decay group, streaming
(master, m, v, grad[, bf16 copy]) once: 16-28 B/param, HBM-bound.
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._ext import native, use_native


def adamw_step_(master: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                lowp: torch.Tensor | None, *, lr: float, beta1: float, beta2: float, eps: float,
                weight_decay: float, step: int, grad_scale=1.0, zero_grad: bool = False) -> None:
    """In-place AdamW on flat 1-D tensors (``grad`` fp32 or bf16).

    ``grad_scale`` is a float or a 1-element f32 device tensor (e.g. the
    grad-clip coefficient x 1/world computed on device: no host sync).
    ``zero_grad``: clear ``grad`` in the same pass (GPU: fused into the kernel)."""
    if use_native(master):
        bc1 = 1.0 - beta1 ** step
        bc2 = 1.0 - beta2 ** step
        if isinstance(grad_scale, torch.Tensor):
            st, sf = grad_scale.reshape(1).float().contiguous(), 1.0
        else:
            st, sf = None, float(grad_scale)
        native().adamw_step(master, grad, m, v, lowp, lr, beta1, beta2, eps, weight_decay, bc1, bc2, st, sf,
                            bool(zero_grad))
        return
    ref.adamw_(master, grad, m, v, lr=lr, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay,
               step=step, grad_scale=grad_scale, p_lowp=lowp)
    if zero_grad:
        grad.zero_()


def sq_norm(x: torch.Tensor) -> torch.Tensor:
    """sum(x^2) as a 1-element fp32 tensor (no host sync).  GPU: one read of x
    (f32 or bf16) with a fixed-order reduction, so every DDP replica computes the
    bitwise-same clip coefficient."""
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous():
        return native().sqnorm(x)
    return x.float().pow(2).sum().reshape(1)
