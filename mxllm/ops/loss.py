"""Fused LM-head + cross-entropy, chunked over T for long sequences.

MI355X-first sizing: at 4k tokens x 128,256 vocab the bf16 logits are 1 GB —
cheap against 288 GB of HBM — so the head runs as ONE large hipBLASLt GEMM
(best MFMA efficiency) instead of many small chunks.  The HIP kernel
``ce_fwd_bwd`` then reads each logits row, computes the loss with an online
log-sum-exp and overwrites the row IN PLACE with d(loss)/d(logits)
(softmax - onehot) / n_valid in bf16.  The backward is a single
``dlogits @ W`` GEMM (plus ``dlogits^T @ h`` when the head is trainable).
``ignore_index`` rows get zero gradient and do not count in the mean.

Long sequences ("chunk over T to avoid materializing"): when the
[T, V] logits would exceed ``MXLLM_CE_CHUNK_GB`` (default 2 GiB: T > 8k tokens
at V = 128,256), the forward walks T in chunks of ``MXLLM_CE_CHUNK_TOKENS``
(default 4096 = 1 GB of bf16 logits) through ONE reused logits buffer: per
chunk the head GEMM, the CE kernel against the GLOBAL valid-token count, and
immediately the chunk's dh rows (dlogits @ W) and its dW contribution (dlogits^T
h into an fp32 accumulator, on the weight-gradient GEMM) — nothing [T, V]-sized
is kept.  The backward only scales dh / dW by the upstream gradient.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import native, use_native
from ..parallel.grad_ready import direct_grad, direct_grad32, mark_ready
from . import gemm
from .linear import param_weight_grad, weight_grad_


def _fp32_logits(chunked: bool) -> bool:
    """MXLLM_CE_FP32_LOGITS: ``chunked`` (default) = the loss of the chunked (long-sequence) path
    is computed from fp32 logits (the head GEMM writes fp32; its bf16 gradient goes to a separate
    buffer), ``1`` = both paths, ``0`` = bf16 logits everywhere (the one-piece path keeps its
    in-place bf16 form by default: +2 GB at T = 4k would sit on the 70B headline's HBM peak)."""
    v = os.environ.get("MXLLM_CE_FP32_LOGITS", "chunked")
    return v == "1" or (v == "chunked" and chunked)


class _LinearCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, labels, ignore_index):
        if _fp32_logits(False):
            lg32 = gemm.mm("tn", h, w, out_dtype=torch.float32)
            logits = torch.empty(lg32.shape, dtype=h.dtype, device=h.device)  # receives dlogits (bf16)
            inv_n = native().ce_inv_count(labels, ignore_index)
            loss = native().ce_chunk_f32(lg32, logits, labels, ignore_index, inv_n).sum() * inv_n[0]
            del lg32
        else:
            logits = gemm.mm("tn", h, w)  # [T, V] bf16
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
            dh = gemm.mm("nn", dlogits, w)
            dh.mul_(gl.to(dh.dtype))  # [T, H]: cheap, unlike scaling the [T, V] dlogits
        if ctx.needs_input_grad[1]:
            # the head's dW: gl folded into dlogits' transpose (token-contiguous operand image)
            dw = param_weight_grad(ctx.wp, dlogits, h, dy_scale=gl)
        return dh, dw, None, None


def _ce_chunk_torch(logits: torch.Tensor, labels: torch.Tensor, inv_n: torch.Tensor, ignore: int) -> torch.Tensor:
    """CPU / reference form of the ce_chunk kernel: per-row losses; ``logits`` <- dlogits * inv_n."""
    lf = logits.float()
    valid = labels != ignore
    lse = torch.logsumexp(lf, dim=-1)
    tgt = lf.gather(1, labels.clamp(min=0).unsqueeze(1)).squeeze(1)
    losses = torch.where(valid, lse - tgt, torch.zeros_like(lse))
    g = torch.softmax(lf, dim=-1)
    g[torch.arange(g.shape[0]), labels.clamp(min=0)] -= 1.0
    g = g * valid.unsqueeze(1).to(g.dtype) * inv_n
    logits.copy_(g.to(logits.dtype))
    return losses


def ce_chunk_tokens(T: int, V: int, elem: int = 2) -> int:
    """Tokens per LM-head chunk for T tokens (T itself = no chunking)."""
    limit = float(os.environ.get("MXLLM_CE_CHUNK_GB", "2")) * 2 ** 30
    if T * V * elem <= limit:
        return T
    return max(1, min(T, int(os.environ.get("MXLLM_CE_CHUNK_TOKENS", "4096"))))


class _ChunkedLinearCEFn(torch.autograd.Function):
    """Mean CE of h @ w^T, T walked in chunks (module doc); dh / dW formed in the forward."""

    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, chunk, grad_mode=True):
        T, V = h.shape[0], w.shape[0]
        nat = use_native(h)
        # gradients are formed here, in the forward: only when a backward can follow (grad mode
        # of the CALLER -- inside forward it is always off -- and an input that requires grad)
        need_h, need_w = grad_mode and ctx.needs_input_grad[0], grad_mode and ctx.needs_input_grad[1]
        if nat:
            inv_n = native().ce_inv_count(labels, ignore_index)
        else:
            inv_n = (1.0 / (labels != ignore_index).sum().clamp(min=1).float()).reshape(1)
        losses = torch.empty(T, dtype=torch.float32, device=h.device)
        dh = torch.empty_like(h) if need_h else None
        dwacc = torch.empty(V, h.shape[1], dtype=torch.float32, device=h.device) if need_w else None
        buf = torch.empty(min(chunk, T), V, dtype=h.dtype, device=h.device)
        f32 = nat and _fp32_logits(True) and h.dtype == torch.bfloat16
        buf32 = torch.empty(min(chunk, T), V, dtype=torch.float32, device=h.device) if f32 else None
        for i, t0 in enumerate(range(0, T, chunk)):
            t1 = min(T, t0 + chunk)
            hc, lab = h[t0:t1], labels[t0:t1]
            lg = buf[: t1 - t0]  # ends as this chunk's bf16 dlogits
            if f32:  # loss from fp32 logits, bf16 gradient into lg
                lg32 = buf32[: t1 - t0]
                gemm.mm("tn", hc, w, out=lg32)
                losses[t0:t1] = native().ce_chunk_f32(lg32, lg, lab, ignore_index, inv_n)
            else:
                gemm.mm("tn", hc, w, out=lg)
                losses[t0:t1] = (native().ce_chunk(lg, lab, ignore_index, inv_n) if nat
                                 else _ce_chunk_torch(lg, lab, inv_n, ignore_index))
            if need_h:
                gemm.mm("nn", lg, w, out=dh[t0:t1])
            if need_w:
                weight_grad_(dwacc, lg, hc, beta=0.0 if i == 0 else 1.0)
        loss = losses.sum() * inv_n[0]
        ctx.save_for_backward(dh, dwacc)
        ctx.wp = w if w.is_leaf else None
        ctx.wdtype = w.dtype
        ctx.scaled = False
        return loss

    @staticmethod
    def backward(ctx, gl):
        dh, dwacc = ctx.saved_tensors
        gdh = gdw = None
        if ctx.needs_input_grad[0]:
            gdh = dh * gl.to(dh.dtype)
        if ctx.needs_input_grad[1]:
            # the fp32 [V, H] accumulator (4 GB at 70B) is scaled in place, so the saved state is
            # consumed: a second backward (retain_graph) would scale it twice -- refuse it
            if ctx.scaled:
                raise RuntimeError("chunked linear_cross_entropy: backward can run only once per forward")
            ctx.scaled = True
            dwacc.mul_(gl)
            wp = ctx.wp
            g = direct_grad(wp) if wp is not None else None
            if g is None and wp is not None:
                g = direct_grad32(wp)
            if g is None:
                gdw = dwacc.to(ctx.wdtype)
            else:
                if getattr(wp, "_mx_grad_fresh", False):
                    g.copy_(dwacc)
                    wp._mx_grad_fresh = False
                else:
                    g.add_(dwacc)
                mark_ready(wp)
        return gdh, gdw, None, None, None, None


def linear_cross_entropy(h: torch.Tensor, w: torch.Tensor, labels: torch.Tensor,
                         ignore_index: int = -100, chunk: int | None = None) -> torch.Tensor:
    """mean CE of ``h @ w.T`` against ``labels`` (h [T,H], w [V,H], labels [T] int64).
    ``chunk``: tokens per LM-head chunk (default: :func:`ce_chunk_tokens`; T = one piece)."""
    T, V = h.shape[0], w.shape[0]
    c = ce_chunk_tokens(T, V) if chunk is None else chunk
    if c < T:
        return _ChunkedLinearCEFn.apply(h.contiguous(), w, labels.contiguous(), ignore_index, c,
                                        torch.is_grad_enabled())
    if use_native(h):
        return _LinearCEFn.apply(h.contiguous(), w, labels.contiguous(), ignore_index)
    return ref.cross_entropy(F.linear(h, w), labels, ignore_index)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Loss only (no grad) on precomputed logits; used for evaluation."""
    if use_native(logits) and logits.dtype == torch.bfloat16:
        loss, _ = native().ce_fwd_bwd(logits.contiguous().clone(), labels.contiguous(), ignore_index)
        return loss
    return ref.cross_entropy(logits, labels, ignore_index)
