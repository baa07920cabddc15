"""Fused LM-head + cross-entropy.

MI355X-first sizing: at 4k tokens x 128,256 vocab the bf16 logits are 1 GB —
cheap against 288 GB of HBM — so the head runs as ONE large hipBLASLt GEMM
(best MFMA efficiency) instead of many small chunks.  The HIP kernel
``ce_fwd_bwd`` then reads each logits row, computes the loss with an online
log-sum-exp and overwrites the row IN PLACE with d(loss)/d(logits)
(softmax - onehot) / n_valid in bf16.  The backward is a single
``dlogits @ W`` GEMM (plus ``dlogits^T @ h`` when the head is trainable).
``ignore_index`` rows get zero gradient and do not count in the mean.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import native, use_native
from .linear import param_weight_grad


class _LinearCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, labels, ignore_index):
        logits = torch.matmul(h, w.t())  # [T, V] bf16, hipBLASLt
        loss, _ = native().ce_fwd_bwd(logits, labels, ignore_index)  # logits <- dlogits
        ctx.save_for_backward(h, w, logits)
        ctx.wp = w if w.is_leaf else None
        return loss

    @staticmethod
    def backward(ctx, gl):
        # the upstream scalar gradient ``gl`` stays on device (no host read to
        # test for 1.0): it scales the small [T, H] dh, and the head's dW through
        # the transpose that forms dlogits' token-contiguous image (no extra pass
        # over the [T, V] dlogits)
        h, w, dlogits = ctx.saved_tensors
        dh = dw = None
        if ctx.needs_input_grad[0]:
            dh = torch.matmul(dlogits, w)
            dh.mul_(gl.to(dh.dtype))  # [T, H]: cheap, unlike scaling the [T, V] dlogits
        if ctx.needs_input_grad[1]:
            # the head's dW: gl folded into dlogits' transpose (token-contiguous operand image)
            dw = param_weight_grad(ctx.wp, dlogits, h, dy_scale=gl)
        return dh, dw, None, None


def linear_cross_entropy(h: torch.Tensor, w: torch.Tensor, labels: torch.Tensor,
                         ignore_index: int = -100) -> torch.Tensor:
    """mean CE of ``h @ w.T`` against ``labels`` (h [T,H], w [V,H], labels [T] int64)."""
    if use_native(h):
        return _LinearCEFn.apply(h.contiguous(), w, labels.contiguous(), ignore_index)
    return ref.cross_entropy(F.linear(h, w), labels, ignore_index)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Loss only (no grad) on precomputed logits; used for evaluation."""
    if use_native(logits) and logits.dtype == torch.bfloat16:
        loss, _ = native().ce_fwd_bwd(logits.contiguous().clone(), labels.contiguous(), ignore_index)
        return loss
    return ref.cross_entropy(logits, labels, ignore_index)
