"""Inference ops: prefill attention into a KV cache, decode attention, sampling.

GPU: csrc/kernels/decode.hip (rope_append, split-K decode attention, Gumbel-max
sampler) and attn_fwd.hip for prefill.  CPU: reference implementations.
"""
from __future__ import annotations

import math

import torch

from . import reference as ref
from ._ext import native, use_native


def prefill_attention(qkv: torch.Tensor, cos, sin, k_cache: torch.Tensor, v_cache: torch.Tensor, slot: int,
                      S: int, Hq: int, Hkv: int, D: int) -> torch.Tensor:
    """One sequence (positions 0..S-1): RoPE, write K/V into ``cache[slot, :, :S]``,
    causal attention.  qkv [S, NH*D] -> o [S, Hq*D]."""
    if use_native(qkv):
        ops = native()
        q, k, v = ops.rope_split(qkv.contiguous(), cos, sin, 1, S, Hq, Hkv, D, None)
        k_cache[slot, :, :S].copy_(k[0])
        v_cache[slot, :, :S].copy_(v[0])
        o, _ = ops.attn_fwd(q, k, v, True, 1.0 / math.sqrt(D))
        return o.view(S, Hq * D)
    x = qkv.view(1, S, Hq + 2 * Hkv, D)
    q = ref.apply_rope(x[:, :, :Hq], cos, sin)
    k = ref.apply_rope(x[:, :, Hq:Hq + Hkv], cos, sin)
    v = x[:, :, Hq + Hkv:]
    k_cache[slot, :, :S].copy_(k[0].transpose(0, 1))
    v_cache[slot, :, :S].copy_(v[0].transpose(0, 1))
    return ref.attention(q, k, v, causal=True).reshape(S, Hq * D)


def decode_attention(qkv: torch.Tensor, cos, sin, k_cache, v_cache, pos: torch.Tensor, slots: torch.Tensor,
                     Hq: int, Hkv: int, D: int, max_len: int) -> torch.Tensor:
    """Batched single-token step.  qkv [B, NH*D], pos/slots int32 [B] (pos = index
    of the new token).  Appends K/V at ``pos`` and attends over ``pos + 1`` keys."""
    if use_native(qkv):
        ops = native()
        q = ops.rope_append(qkv.contiguous(), cos, sin, pos, slots, k_cache, v_cache, Hq, Hkv, D)
        return ops.decode_attn(q, k_cache, v_cache, pos, slots, max_len, 1.0 / math.sqrt(D), 1)
    B = qkv.shape[0]
    x = qkv.view(B, Hq + 2 * Hkv, D).float()
    outs = []
    for i in range(B):
        p, s = int(pos[i]), int(slots[i])
        c = cos[p].view(1, D // 2)
        sn = sin[p].view(1, D // 2)

        def rot(t):
            t1, t2 = t[..., : D // 2], t[..., D // 2:]
            return torch.cat([t1 * c - t2 * sn, t2 * c + t1 * sn], -1)

        qi = rot(x[i, :Hq])
        ki = rot(x[i, Hq:Hq + Hkv])
        k_cache[s, :, p] = ki.to(k_cache.dtype)
        v_cache[s, :, p] = x[i, Hq + Hkv:].to(v_cache.dtype)
        kk = k_cache[s, :, :p + 1].float().repeat_interleave(Hq // Hkv, 0)  # [Hq, L, D]
        vv = v_cache[s, :, :p + 1].float().repeat_interleave(Hq // Hkv, 0)
        sc = torch.einsum("hd,hld->hl", qi, kk) / math.sqrt(D)
        outs.append(torch.einsum("hl,hld->hd", sc.softmax(-1), vv).reshape(-1))
    return torch.stack(outs).to(qkv.dtype)


def sample(logits: torch.Tensor, temperature: float = 0.0, seed: int = 0, step: int = 0,
           top_p: float = 1.0, top_k: int = 0) -> torch.Tensor:
    """logits [B, V] -> token ids [B] int64.  Greedy when temperature <= 0.
    Temperature sampling is exact (Gumbel-max) in one pass on GPU; top-k /
    top-p first mask the logits (torch sort) then sample the same way."""
    if top_k > 0 or top_p < 1.0:
        logits = _mask_top(logits.float(), top_k, top_p)
    if use_native(logits):
        return native().sample(logits.contiguous(), float(temperature), int(seed), int(step))
    if temperature <= 0:
        return logits.float().argmax(-1)
    g = torch.Generator(device=logits.device)
    g.manual_seed(seed * 1000003 + step)
    probs = torch.softmax(logits.float() / temperature, -1)
    return torch.multinomial(probs, 1, generator=g).view(-1)


def _mask_top(logits: torch.Tensor, top_k: int, top_p: float) -> torch.Tensor:
    if top_k > 0:
        kth = torch.topk(logits, min(top_k, logits.shape[-1]), -1).values[..., -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p < 1.0:
        srt, idx = torch.sort(logits, -1, descending=True)
        cp = torch.softmax(srt, -1).cumsum(-1)
        drop = cp - torch.softmax(srt, -1) > top_p
        srt = srt.masked_fill(drop, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, idx, srt)
    return logits
