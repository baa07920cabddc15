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
            [B,Hq,S,D] f32 --rope_merge_bwd--> d(qkv) bf16 [T,(Hq+2Hkv)D]; at D = 128 the
            dQ kernel writes d(q) of d(qkv) itself (attn_bwd_rope, backward_dqkv)
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
        dqkv = backward_dqkv(do, q, k, v, o, lse, cos, sin, causal, grad_pad)
        return dqkv, None, None, None, None, None, None, None, None, None, None


_DS_BUDGET = float(os.environ.get("MXLLM_ATTN_DS_BUDGET_GB", "4")) * 2**30


def _ds_bytes_per_head(S: int, Sk: int) -> int:
    return (Sk + 127) // 128 * 128 * ((S + 63) // 64 * 64) * 2


def backward_dqkv(do, q, k, v, o, lse, cos, sin, causal: bool, grad_pad: int = 0) -> torch.Tensor:
    """d(qkv) [B*S, (Hq+2Hkv)*D (+grad_pad)] bf16 of the RoPE'd attention block.  The split backward at
    D = 128 writes it directly (``attn_bwd_rope``: the dQ kernel applies the inverse RoPE to d(q) and
    rounds once, rope_merge_bwd fills only the k / v columns; no fp32 dQ through HBM -- 70B training
    shape: -201 MB of traffic per layer); otherwise fp32 dQ + dK / dV partials then rope_merge_bwd.
    ``MXLLM_ATTN_DQ_ROPE=0`` forces the two-step path (A/B)."""
    ops = native()
    B, Hq, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    scale = 1.0 / math.sqrt(D)
    mode = dq_mode()
    if (mode == 3 and D == 128 and Sk == S and B * Hq * _ds_bytes_per_head(S, Sk) <= _DS_BUDGET
            and os.environ.get("MXLLM_ATTN_DQ_ROPE", "1") != "0"):
        return ops.attn_bwd_rope(do.contiguous(), q, k, v, o, lse, causal, scale, cos, sin, grad_pad)
    dq, dkp, dvp = attn_bwd(do.contiguous(), q, k, v, o, lse, causal, scale, mode)
    return ops.rope_merge_bwd(dq, dkp, dvp, cos, sin, B, S, Hq, Hkv, D, grad_pad)


def attn_bwd(do, q, k, v, o, lse, causal: bool, scale: float, mode: int):
    """``native().attn_bwd`` with bounded memory.  The split dQ mode (3) passes dS^T through an
    HBM image of B * Hq * Sk * S bf16 -- O(S^2): 1.1 GB at the 70B training shape, 64 GiB for one
    8B sequence of 32k tokens.  Above ``MXLLM_ATTN_DS_BUDGET_GB`` (4 GiB) the call runs per
    (sequence, chunk of whole KV groups), each chunk's image within the budget, writing its dQ and
    dK / dV partials into head ranges of the full outputs (a KV head's partials stay consecutive for
    rope_merge_bwd).
    ``do`` [B*S, Hq*D] or [B, S, Hq*D], ``o`` [B, S, Hq*D] (row-strided allowed)."""
    ops = native()
    B, Hq, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    per_head = _ds_bytes_per_head(S, Sk)
    if mode != 3 or B * Hq * per_head <= _DS_BUDGET:
        return ops.attn_bwd(do, q, k, v, o, lse, causal, scale, mode)
    G = Hq // Hkv
    hpc = G  # heads per chunk: whole KV groups, a divisor of Hq (equal chunks -> equal partial layout)
    for c in range(G, Hq + 1, G):
        if Hq % c == 0 and c * per_head <= _DS_BUDGET:
            hpc = c
    do4 = do.reshape(B, S, Hq, D)
    o3 = o.view(B, S, o.shape[-1]) if o.dim() != 3 else o
    n = Hq // hpc
    dq = dk = dv = None
    for b in range(B):
        for i in range(n):
            h0, h1 = i * hpc, (i + 1) * hpc
            args = (do4[b:b + 1, :, h0:h1].contiguous(), q[b:b + 1, h0:h1], k[b:b + 1, h0 // G:h1 // G],
                    v[b:b + 1, h0 // G:h1 // G], o3[b:b + 1, :, h0 * D:h1 * D], lse[b:b + 1, h0:h1], causal, scale, 3)
            if dq is None:  # first chunk: its partial-head count sizes the full dK / dV partials
                dq_c, dk_c, dv_c = ops.attn_bwd(*args)
                P = dk_c.shape[1]
                dq = torch.empty(B, Hq, S, D, dtype=dq_c.dtype, device=dq_c.device)
                dk = torch.empty(B, n * P, Sk, D, dtype=dk_c.dtype, device=dk_c.device)
                dv = torch.empty_like(dk)
                dq[0:1, h0:h1].copy_(dq_c)
                dk[0:1, 0:P].copy_(dk_c)
                dv[0:1, 0:P].copy_(dv_c)
                del dq_c, dk_c, dv_c
            else:  # every other chunk writes its head range in place
                ops.attn_bwd(*args, dq[b:b + 1, h0:h1], dk[b:b + 1, i * P:(i + 1) * P], dv[b:b + 1, i * P:(i + 1) * P])
    return dq, dk, dv


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
