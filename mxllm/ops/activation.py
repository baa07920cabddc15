"""SwiGLU ``silu(gate) * up`` over a fused [gate | up] projection.

GPU: csrc/kernels/swiglu.hip (vectorised 16-B bf16, fwd + bwd in one pass each).
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._ext import native, use_native


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dm):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(dm.contiguous(), gu)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    if use_native(gate_up):
        return _SwiGLUFn.apply(gate_up.contiguous())
    return ref.swiglu(gate_up)
