"""Fused attention block: QKV split + Llama-3 RoPE + causal GQA flash attention.

SURVEY §2.4 K6 + K7 (+K13 prefill).  The whole ``qkv -> o`` segment is ONE
autograd node so the backward can hand the attention kernel's f32 dQ and
per-q-head dK/dV partials straight to the inverse-RoPE merge kernel, which
writes d(qkv) in the projection's token-major layout — no intermediate
re-layout tensors and no autograd shape constraints between them.

GPU path (csrc/kernels/rope.hip, attn_fwd.hip, attn_bwd.hip):
  forward : qkv [T,(Hq+2Hkv)D] --rope_split--> q [B,Hq,S,D], k,v [B,Hkv,S,D]
            --attn_fwd (MFMA 32x32x16 bf16)--> o [B,S,Hq*D] token-major, lse [B,Hq,S]
  backward: attn_bwd -> dq f32 [B,Hq,S,D] (dS^T through HBM + a dQ kernel by
            default; f32-atomic and partial-sum modes selectable), dk/dv partials
            [B,Hq,S,D] f32 --rope_merge_bwd--> d(qkv) bf16 [T,(Hq+2Hkv)D]
"""
from __future__ import annotations

import math
import os

import torch

from . import reference as ref
from ._ext import native, use_native


def split_heads_ref(qkv: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, D: int):
    x = qkv.view(B, S, Hq + 2 * Hkv, D)
    return x[:, :, :Hq], x[:, :, Hq:Hq + Hkv], x[:, :, Hq + Hkv:]


class _AttnBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, Hq, Hkv, D, causal, out_pad, grad_pad):
        ops = native()
        q, k, v = ops.rope_split(qkv, cos, sin, B, S, Hq, Hkv, D)
        o, lse = ops.attn_fwd(q, k, v, causal, 1.0 / math.sqrt(D), out_pad)
        ctx.save_for_backward(q, k, v, o, lse, cos, sin)
        ctx.dims = (B, S, Hq, Hkv, D, causal, grad_pad)
        return o.view(B * S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cos, sin = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, grad_pad = ctx.dims
        ops = native()
        dq, dkp, dvp = ops.attn_bwd(do.contiguous(), q, k, v, o, lse, causal, 1.0 / math.sqrt(D), dq_mode())
        dqkv = ops.rope_merge_bwd(dq, dkp, dvp, cos, sin, B, S, Hq, Hkv, D, grad_pad)
        return dqkv, None, None, None, None, None, None, None, None, None, None


def dq_mode() -> int:
    """How the attention backward forms dQ (csrc/kernels/attn_bwd.hip):
    3 = split (dS^T to HBM, separate dQ kernel; fastest and deterministic, default),
    2 = per-key-block partials + ordered reduction, 1 = f32 atomics (non-deterministic).
    ``MXLLM_ATTN_DQ_MODE`` overrides; with ``torch.use_deterministic_algorithms(True)``
    or ``MXLLM_DETERMINISTIC=1`` mode 1 is never used."""
    m = int(os.environ.get("MXLLM_ATTN_DQ_MODE", "3"))
    if m == 1 and (torch.are_deterministic_algorithms_enabled() or os.environ.get("MXLLM_DETERMINISTIC") == "1"):
        m = 3
    return m


def attention_block(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, B: int, S: int, Hq: int,
                    Hkv: int, D: int, causal: bool = True, out_pad: int = 0, grad_pad: int = 0) -> torch.Tensor:
    """qkv [B*S, (Hq+2Hkv)*D] -> attention output [B*S, Hq*D] (RoPE at positions 0..S-1).
    ``out_pad`` / ``grad_pad``: padded row layouts of the output and of d(qkv)
    for LoRA-augmented GEMM neighbours (mxllm/ops/linear.py)."""
    if use_native(qkv):
        return _AttnBlockFn.apply(qkv.contiguous(), cos, sin, B, S, Hq, Hkv, D, causal, out_pad, grad_pad)
    q, k, v = split_heads_ref(qkv, B, S, Hq, Hkv, D)
    q = ref.apply_rope(q, cos, sin)
    k = ref.apply_rope(k, cos, sin)
    o = ref.attention(q, k, v, causal=causal)
    return o.reshape(B * S, Hq * D)
