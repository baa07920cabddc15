"""Token embedding gather / scatter-add.

GPU: csrc/kernels/embedding.hip — forward is a 16-B-vectorised row gather
(one wave per token row); backward adds rows into an f32 [V, H] accumulator
with no-return f32 atomics shaped as full 256-B wave instructions (the chip's
atomic path runs at ~1.3 TB/s, far above what 4k-token steps need), then
casts to the parameter dtype.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..parallel.grad_ready import accum_grad, deliver_grad
from ._ext import native, use_native


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.vocab = weight.shape[0]
        ctx.wdtype = weight.dtype
        ctx.wp = weight if weight.is_leaf else None  # for an owner-side gradient sink (ZeRO-3)
        ctx.nat = use_native(weight)
        return native().embedding_fwd(ids, weight) if ctx.nat else F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None
        if ctx.nat:
            dw = native().embedding_bwd(dy.contiguous(), ids, ctx.vocab)  # f32 accumulator
        else:
            dy2 = dy.reshape(-1, dy.shape[-1])
            dw = torch.zeros(ctx.vocab, dy2.shape[1], dtype=torch.float32, device=dy.device)
            dw.index_add_(0, ids.reshape(-1), dy2.float())
        # fp32 gradient owners take the f32 sums as they are (no bf16 rounding)
        if accum_grad(ctx.wp, dw):
            return None, None
        sink32 = getattr(ctx.wp, "_mx_grad_sink_dtype", None) == torch.float32
        if deliver_grad(ctx.wp, dw if sink32 else dw.to(ctx.wdtype)):
            return None, None
        return None, dw.to(ctx.wdtype)


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if use_native(weight) or getattr(weight, "_mx_grad_sink", None) is not None:
        return _EmbeddingFn.apply(ids.contiguous(), weight)
    return F.embedding(ids, weight)
