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


class SplitMaster:
    """fp32 master weights stored as two 16-bit halves of their bit pattern:
    ``hi`` — the bf16 COMPUTE weights themselves (the master rounded half-up on its
    bits) — and ``lo`` (int16) = master bits - (hi << 16), which always fits.  The
    fp32 value is reconstructed exactly, so the optimizer arithmetic is that of an
    fp32 master; the separate bf16 copy disappears: 2 B/param less optimizer state
    (8B full fine-tune: 16 GB; a 70B ZeRO-3 rank at world 8: 17.6 GB) and 2 B/param
    less AdamW traffic.  Only exact ties round differently from round-to-nearest-even.

    Behaves like a 1-D fp32 tensor where the framework needs one: slicing (views of
    both halves), ``copy_`` (split), ``zero_``, and ``float()`` / ``detach()`` /
    ``contiguous()`` / ``cpu()`` / ``clone()`` / ``view()`` (a materialised fp32
    copy, for checkpoints, tests and export)."""

    dtype = torch.float32

    def __init__(self, hi: torch.Tensor, lo: torch.Tensor | None = None):
        self.hi = hi
        self.lo = lo if lo is not None else torch.zeros(hi.shape, dtype=torch.int16, device=hi.device)

    @property
    def device(self):
        return self.hi.device

    @property
    def shape(self):
        return self.hi.shape

    @property
    def is_cuda(self):
        return self.hi.is_cuda

    def numel(self) -> int:
        return self.hi.numel()

    def element_size(self) -> int:
        return 4

    def storage_offset(self) -> int:
        return self.hi.storage_offset()

    def __getitem__(self, sl):
        return SplitMaster(self.hi[sl], self.lo[sl])

    def float(self) -> torch.Tensor:
        out = torch.empty(self.hi.shape, dtype=torch.float32, device=self.hi.device)
        if use_native(self.hi) and self.hi.is_contiguous() and self.lo.is_contiguous():
            native().join_master(self.hi, self.lo, out)
            return out
        b = (self.hi.view(torch.int16).to(torch.int64) & 0xFFFF) << 16
        b = (b + self.lo.to(torch.int64)) & 0xFFFFFFFF
        b = torch.where(b >= 2 ** 31, b - 2 ** 32, b)
        out.copy_(b.to(torch.int32).view(torch.float32))
        return out

    def detach(self):
        return self.float()

    contiguous = clone = detach

    def cpu(self):
        return self.float().cpu()

    def view(self, *shape):
        return self.float().view(*shape)

    def zero_(self):
        self.hi.zero_()
        self.lo.zero_()
        return self

    def copy_(self, src: torch.Tensor):
        x = src.to(device=self.hi.device, dtype=torch.float32).reshape(self.hi.shape).contiguous()
        if use_native(self.hi) and self.hi.is_contiguous() and self.lo.is_contiguous():
            native().split_master(x, self.hi, self.lo)
            return self
        b = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        h = ((b + 0x8000) >> 16) & 0xFFFF
        lo = b - (h << 16)
        lo = torch.where(lo >= 2 ** 31, lo - 2 ** 32, lo)  # h << 16 wrapped past 2^32 (negative numbers)
        self.lo.copy_(lo.to(torch.int16))
        self.hi.view(torch.int16).copy_(torch.where(h >= 2 ** 15, h - 2 ** 16, h).to(torch.int16))
        return self


def adamw_step_(master, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                lowp: torch.Tensor | None, *, lr: float, beta1: float, beta2: float, eps: float,
                weight_decay: float, step: int, grad_scale=1.0, zero_grad: bool = False) -> None:
    """In-place AdamW on flat 1-D tensors (``grad`` fp32 or bf16).

    ``master``: an fp32 tensor (``lowp``: optional bf16 copy to refresh) or a
    :class:`SplitMaster` (its ``hi`` half IS the bf16 copy; ``lowp`` ignored).
    ``grad_scale`` is a float or a 1-element f32 device tensor (e.g. the
    grad-clip coefficient x 1/world computed on device: no host sync).
    ``zero_grad``: clear ``grad`` in the same pass (GPU: fused into the kernel)."""
    split = isinstance(master, SplitMaster)
    if use_native(m):
        bc1 = 1.0 - beta1 ** step
        bc2 = 1.0 - beta2 ** step
        if isinstance(grad_scale, torch.Tensor):
            st, sf = grad_scale.reshape(1).float().contiguous(), 1.0
        else:
            st, sf = None, float(grad_scale)
        if split:
            native().adamw_step(None, grad, m, v, master.hi, master.lo, lr, beta1, beta2, eps, weight_decay, bc1,
                                bc2, st, sf, bool(zero_grad))
        else:
            native().adamw_step(master, grad, m, v, lowp, None, lr, beta1, beta2, eps, weight_decay, bc1, bc2, st,
                                sf, bool(zero_grad))
        return
    p = master.float() if split else master
    ref.adamw_(p, grad, m, v, lr=lr, beta1=beta1, beta2=beta2, eps=eps, weight_decay=weight_decay,
               step=step, grad_scale=grad_scale, p_lowp=None if split else lowp)
    if split:
        master.copy_(p)
    if zero_grad:
        grad.zero_()


def sq_norm(x: torch.Tensor) -> torch.Tensor:
    """sum(x^2) as a 1-element fp32 tensor (no host sync).  GPU: one read of x
    (f32 or bf16) with a fixed-order reduction, so every DDP replica computes the
    bitwise-same clip coefficient."""
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous():
        return native().sqnorm(x)
    return x.float().pow(2).sum().reshape(1)
