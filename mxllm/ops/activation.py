"""SwiGLU ``silu(gate) * up`` over a fused [gate | up] projection.

GPU: csrc/kernels/elementwise.hip ``swiglu_fwd_kernel`` / ``swiglu_bwd_kernel`` (vectorised 16-B
bf16, fwd + bwd in one pass each).
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._ext import native, use_native


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, out_pad, grad_pad):
        ctx.save_for_backward(gu)
        ctx.grad_pad = grad_pad
        return native().swiglu_fwd(gu, out_pad)

    @staticmethod
    def backward(ctx, dm):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(dm.contiguous(), gu, ctx.grad_pad), None, None


def swiglu(gate_up: torch.Tensor, out_pad: int = 0, grad_pad: int = 0) -> torch.Tensor:
    """``out_pad`` / ``grad_pad``: padded row layouts for LoRA-augmented GEMM
    neighbours (see mxllm/ops/norm.py)."""
    if use_native(gate_up):
        if gate_up.dim() != 2:
            out_pad = grad_pad = 0
        return _SwiGLUFn.apply(gate_up.contiguous(), out_pad, grad_pad)
    return ref.swiglu(gate_up)
