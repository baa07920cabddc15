"""SwiGLU ``silu(gate) * up`` over a fused [gate | up] projection.

GPU: csrc/kernels/elementwise.hip ``swiglu_fwd_kernel`` / ``swiglu_bwd_kernel`` (vectorised 16-B
bf16, fwd + bwd in one pass each).  Next to LoRA-augmented projections (mxllm/ops/linear.py
``_LoRAAugFn``) the same pass can also produce the neighbour's rank-r tail
(csrc/kernels/lora.hip ``swiglu_lora_kernel``): forward ``s m A_down^T`` into the pad columns of
``m``, backward ``s dgu B_gu`` into the pad columns of ``dgu`` -- the down projection's input and
the gate-up projection's output gradient are then never re-read for their LoRA products.
"""
from __future__ import annotations

import os

import torch

from . import reference as ref
from ._ext import native, use_native


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, out_pad, grad_pad, tail_fwd, tail_bwd):
        ctx.save_for_backward(gu)
        ctx.grad_pad = grad_pad
        ctx.tail_bwd = tail_bwd
        if tail_fwd is not None:
            v, nrb, s = tail_fwd
            return native().swiglu_lora(None, gu, out_pad, v, nrb, s)
        return native().swiglu_fwd(gu, out_pad)

    @staticmethod
    def backward(ctx, dm):
        (gu,) = ctx.saved_tensors
        if ctx.tail_bwd is not None:
            v, nrb, s = ctx.tail_bwd
            dgu = native().swiglu_lora(dm.contiguous(), gu, ctx.grad_pad, v, nrb, s)
        else:
            dgu = native().swiglu_bwd(dm.contiguous(), gu, ctx.grad_pad)
        return dgu, None, None, None, None


def lora_tail_ok(x: torch.Tensor, T: int, F2: int, pad: int, R: int) -> bool:
    """Whether the fused SwiGLU + LoRA-tail kernel takes a [T, F2] gate-up projection on
    ``x``'s device / dtype (``R`` = the neighbour's n * r, ``pad`` its augmented-buffer padding)."""
    return (_FUSE_TAIL and use_native(x) and x.dtype == torch.bfloat16 and T % 16 == 0 and F2 % 256 == 0
            and R % 16 == 0 and 16 <= R <= 64 and R <= pad and pad % 8 == 0)


_FUSE_TAIL = os.environ.get("MXLLM_SWIGLU_LORA", "1") != "0"  # A/B switch


def swiglu(gate_up: torch.Tensor, out_pad: int = 0, grad_pad: int = 0, tail_fwd=None, tail_bwd=None) -> torch.Tensor:
    """``out_pad`` / ``grad_pad``: padded row layouts for LoRA-augmented GEMM
    neighbours (see mxllm/ops/norm.py).  ``tail_fwd`` = (V [>= R, F] row view, R, s): also write
    ``s m V^T`` into the ``out_pad`` columns; ``tail_bwd`` = (V [>= R, 2F], R, s): write
    ``s dgu V^T`` into the ``grad_pad`` columns of the input gradient (callers check
    ``lora_tail_ok`` first)."""
    if use_native(gate_up):
        if gate_up.dim() != 2:
            out_pad = grad_pad = 0
            tail_fwd = tail_bwd = None
        tf = (tail_fwd[0], tail_fwd[1] // 16, float(tail_fwd[2])) if tail_fwd is not None else None
        tb = (tail_bwd[0], tail_bwd[1] // 16, float(tail_bwd[2])) if tail_bwd is not None else None
        return _SwiGLUFn.apply(gate_up.contiguous(), out_pad, grad_pad, tf, tb)
    return ref.swiglu(gate_up)
