"""Linear layers: plain (hipBLASLt via torch.matmul) and fused multi-adapter LoRA.

A fused projection (e.g. Wqkv = [Wq; Wk; Wv], Wgu = [Wg; Wu]) carries one
LoRA adapter per output split.  All splits share the input, so their A
matrices are concatenated into one ``A_cat [n*r, in]`` and the down-projection
``t = x @ A_cat^T`` is ONE skinny GEMM; each split's up-projection
``y[:, split_i] += s * t_i @ B_i^T`` is written straight into the column
slice of the base GEMM's output (hipBLASLt handles the leading dimension).

Backward (base weight frozen — its gradient is never formed):
  g_i  = s * dy_i @ B_i          dB_i = s * dy_i^T @ t_i
  dA   = g^T @ x                 dx   = dy @ W + g @ A_cat
Only ``x`` and the tiny ``t`` are saved.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn.functional as F


class _LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, a_cat, scaling, splits, *bs):
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.matmul(x2, w.t())
        a = a_cat.to(x.dtype)
        t = torch.matmul(x2, a.t())  # [T, n*r]
        r = a_cat.shape[0] // len(bs)
        off = 0
        for i, (n_i, b) in enumerate(zip(splits, bs)):
            y[:, off:off + n_i].addmm_(t[:, i * r:(i + 1) * r], b.to(x.dtype).t(), alpha=scaling)
            off += n_i
        ctx.save_for_backward(x2, w, a_cat, t, *bs)
        ctx.scaling, ctx.splits, ctx.r = scaling, tuple(splits), r
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, a_cat, t, *bs = ctx.saved_tensors
        s, r = ctx.scaling, ctx.r
        dy2 = dy.reshape(-1, dy.shape[-1])
        dt = x2.dtype
        g = torch.empty(dy2.shape[0], a_cat.shape[0], dtype=dt, device=dy.device)
        dbs = []
        off = 0
        for i, (n_i, b) in enumerate(zip(ctx.splits, bs)):
            dyi = dy2[:, off:off + n_i]
            torch.matmul(dyi, b.to(dt), out=g[:, i * r:(i + 1) * r])
            if s != 1.0:
                g[:, i * r:(i + 1) * r].mul_(s)
            dbs.append((torch.matmul(dyi.t(), t[:, i * r:(i + 1) * r]) * s).to(b.dtype))
            off += n_i
        da = torch.matmul(g.t(), x2).to(a_cat.dtype)
        dx = torch.matmul(dy2, w)
        dx.addmm_(g, a_cat.to(dt))
        return (dx.view(ctx.xshape), None, da, None, None, *dbs)


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return F.linear(x, w)


def lora_linear(x: torch.Tensor, w: torch.Tensor, a_cat: torch.Tensor, bs: Sequence[torch.Tensor],
                splits: Sequence[int], scaling: float) -> torch.Tensor:
    return _LoRALinearFn.apply(x, w, a_cat, scaling, tuple(splits), *bs)
