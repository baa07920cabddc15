"""Linear layers: plain (hipBLASLt via torch.matmul) and fused multi-adapter LoRA.

A fused projection (Wqkv = [Wq; Wk; Wv], Wgu = [Wg; Wu]) carries one LoRA
adapter of rank r per output split.  All splits share the input, so
  * A is one [n*r, in] matrix: the down-projection t = x A^T is ONE skinny GEMM;
  * B is one BLOCK-DIAGONAL [N, n*r] matrix (split i's B_i in rows of split i,
    columns i*r..(i+1)*r; zeros elsewhere, never updated because their
    gradient is written as exact zeros): the up-projection is ONE GEMM.
Adapters are bf16 compute weights (fp32 master + Adam state live in the
flat optimizer buffers), so no per-call casts.

MI355X/hipBLASLt fusion: the LoRA term is not added with a separate
read-modify-write of the (huge) projection output.  It is written first and
then consumed as the C input of the base GEMM (beta = 1), whose epilogue reads
it while the GEMM is compute-bound (measured: beta=1 runs at the same
TFLOP/s as beta=0 on every Llama-3.1 projection shape):
  forward : y  = s t B^T            ; y  += x  W^T   (base GEMM, C = y)
  backward: g  = s dy B             ; dx  = g A      ; dx += dy W (base GEMM, C = dx)
            dB_i = s dy_i^T t_i (diagonal blocks only) ; dA = g^T x
Only x and the tiny t are saved for backward; the frozen base weight's
gradient is never formed.  The LoRA scale rides in the GEMM alpha, and when
the trainer has pre-attached flat .grad buffers the adapter gradients are
accumulated into them by the GEMMs themselves (beta = 1) — no zero-fill,
cast or accumulate kernels — and DDP is told via ``mark_ready``.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn.functional as F

from ..parallel.grad_ready import direct_grad, mark_ready


class _LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, a, b, scaling, splits, r):
        x2 = x.reshape(-1, x.shape[-1])
        t = torch.matmul(x2, a.t())  # [T, n*r]
        y = torch.empty(x2.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        y.addmm_(t, b.t(), beta=0.0, alpha=scaling)  # LoRA term first (scale folded into alpha) ...
        y.addmm_(x2, w.t())  # ... then the base GEMM with C = y (beta = 1)
        ctx.save_for_backward(x2, w, a, b, t)
        ctx.scaling, ctx.splits, ctx.r, ctx.xshape = scaling, tuple(splits), r, x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, a, b, t = ctx.saved_tensors
        s, r = ctx.scaling, ctx.r
        dy2 = dy.reshape(-1, dy.shape[-1])
        g = torch.empty(dy2.shape[0], a.shape[0], dtype=dy2.dtype, device=dy2.device)
        g.addmm_(dy2, b, beta=0.0, alpha=s)  # [T, n*r] (block-diagonal B)
        # adapter grads: accumulate straight into the (flat) .grad buffers when
        # they exist (trainer-managed), otherwise hand them to autograd
        ga, gb = direct_grad(a) if ctx.needs_input_grad[2] else None, direct_grad(b) if ctx.needs_input_grad[3] else None
        da = db = None
        if ctx.needs_input_grad[2]:
            if ga is not None:
                ga.addmm_(g.t(), x2)
                mark_ready(a)
            else:
                da = torch.matmul(g.t(), x2)
        if ctx.needs_input_grad[3]:
            tgt = gb if gb is not None else torch.zeros_like(b)
            off = 0
            for i, n_i in enumerate(ctx.splits):
                tgt[off:off + n_i, i * r:(i + 1) * r].addmm_(dy2[:, off:off + n_i].t(), t[:, i * r:(i + 1) * r],
                                                            beta=1.0 if gb is not None else 0.0, alpha=s)
                off += n_i
            if gb is not None:
                mark_ready(b)
            else:
                db = tgt
        dx = torch.matmul(g, a)
        dx.addmm_(dy2, w)  # base dX GEMM with C = g A (beta = 1)
        return dx.view(ctx.xshape), None, da, db, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return F.linear(x, w)


def lora_linear(x: torch.Tensor, w: torch.Tensor, a: torch.Tensor, b: torch.Tensor, splits: Sequence[int],
                scaling: float) -> torch.Tensor:
    """y = x W^T + scaling * (x A^T) Bbd^T with block-diagonal Bbd (see module doc)."""
    r = a.shape[0] // len(splits)
    return _LoRALinearFn.apply(x, w, a, b, scaling, tuple(splits), r)
