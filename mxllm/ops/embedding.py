"""Token embedding gather / scatter-add.

GPU: csrc/kernels/elementwise.hip — forward is a 16-B-vectorised row gather
(one wave per token row).  Backward, when the parameter's owner exposes its
gradient buffer (DDP flat grads, bf16 or fp32): the batch's ids are stably
sorted and one workgroup per distinct id sums its dy rows in fp32 and adds them
into that row of the buffer (touched rows only, deterministic).  Otherwise: rows
added into an f32 [V, H] accumulator with no-return f32 atomics (256-B wave
instructions), then cast to the parameter dtype.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import os

from ..parallel.grad_ready import accum_grad, deliver_grad, direct_grad, direct_grad32, mark_ready
from ._ext import native, use_native

# sparse backward straight into the owner's gradient buffer (touched rows only); 0 = the
# dense f32 accumulator path (A/B)
_SPARSE_BWD = os.environ.get("MXLLM_EMB_SPARSE_BWD", "1") != "0"


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
        if ctx.nat and _SPARSE_BWD and ctx.wp is not None:
            # the owner's buffer (fp32 accumulation target, else the preallocated .grad):
            # zero it when this is the step's first write, then add only the rows of the
            # batch's tokens, each summed over its occurrences in a fixed order
            t = direct_grad32(ctx.wp)
            if t is None:
                t = direct_grad(ctx.wp)
            if t is not None and t.is_contiguous() and t.dim() == 2:
                if getattr(ctx.wp, "_mx_grad_fresh", False):
                    t.zero_()
                    ctx.wp._mx_grad_fresh = False
                sid, perm = torch.sort(ids.reshape(-1), stable=True)
                native().embedding_bwd_sorted(dy.reshape(-1, dy.shape[-1]).contiguous(), sid, perm, t)
                mark_ready(ctx.wp)
                return None, None
        if ctx.nat and _SPARSE_BWD:
            # no owner buffer (e.g. tied embeddings: autograd sums this with the head's gradient):
            # the same sorted, fixed-order row sums into a zeroed f32 [V, H] -- deterministic, unlike
            # the atomic accumulator below (its fp32 add order varies run to run)
            dw = torch.zeros(ctx.vocab, dy.shape[-1], dtype=torch.float32, device=dy.device)
            sid, perm = torch.sort(ids.reshape(-1), stable=True)
            native().embedding_bwd_sorted(dy.reshape(-1, dy.shape[-1]).contiguous(), sid, perm, dw)
        elif ctx.nat:
            dw = native().embedding_bwd(dy.contiguous(), ids, ctx.vocab)  # f32 accumulator (atomics)
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
