"""Inference ops: prefill attention into a KV cache, decode attention, sampling.

GPU: csrc/kernels/decode.hip (rope_append, split-K decode attention, greedy /
Gumbel-max sampler), sampling.hip (batched top-k / top-p / temperature) and
attn_fwd.hip for prefill.  CPU: reference implementations.
"""
from __future__ import annotations

import math

import torch

from . import reference as ref
from ._ext import native, use_native


def prefill_attention(qkv: torch.Tensor, cos, sin, write_kv, S: int, Hq: int, Hkv: int, D: int) -> torch.Tensor:
    """One sequence (positions 0..S-1): RoPE, hand the rotated K and V [Hkv, S, D] to
    ``write_kv(k, v)`` (the engine's KV cache), causal attention.
    qkv [S, NH*D] -> o [S, Hq*D]."""
    if use_native(qkv):
        ops = native()
        q, k, v = ops.rope_split(qkv.contiguous(), cos, sin, 1, S, Hq, Hkv, D, None)
        write_kv(k[0], v[0])
        o, _ = ops.attn_fwd(q, k, v, True, 1.0 / math.sqrt(D))
        return o.view(S, Hq * D)
    x = qkv.view(1, S, Hq + 2 * Hkv, D)
    q = ref.apply_rope(x[:, :, :Hq], cos, sin)
    k = ref.apply_rope(x[:, :, Hq:Hq + Hkv], cos, sin)
    v = x[:, :, Hq + Hkv:]
    write_kv(k[0].transpose(0, 1), v[0].transpose(0, 1))
    return ref.attention(q, k, v, causal=True).reshape(S, Hq * D)


def _kv_at(cache: torch.Tensor, bt, slot: int, p0: int, p1: int) -> torch.Tensor:
    """Rows [p0, p1) of ``slot`` as [Hkv, p1 - p0, D] (contiguous or paged cache; a view
    when they lie in one block)."""
    if bt is None:
        return cache[slot, :, p0:p1]
    blk = cache.shape[2]
    if p0 // blk == (p1 - 1) // blk:
        b = int(bt[slot, p0 // blk])
        return cache[b, :, p0 % blk:p0 % blk + (p1 - p0)]
    parts, a = [], p0
    while a < p1:
        e = min(p1, (a // blk + 1) * blk)
        parts.append(_kv_at(cache, bt, slot, a, e))
        a = e
    return torch.cat(parts, 1)


def decode_attention(qkv: torch.Tensor, cos, sin, k_cache, v_cache, pos: torch.Tensor, slots: torch.Tensor,
                     Hq: int, Hkv: int, D: int, max_len: int, block_table: torch.Tensor | None = None,
                     counters: torch.Tensor | None = None) -> torch.Tensor:
    """Batched single-token step.  qkv [B, NH*D], pos/slots int32 [B] (pos = index
    of the new token).  Appends K/V at ``pos`` and attends over ``pos + 1`` keys.
    ``block_table`` [slots, max_blocks] int32: paged caches [blocks, Hkv, block, D].
    ``counters``: zeroed int32 [>= B * Hkv] owned by the caller — the split-K
    partials then merge inside the attention launch (no combine kernel)."""
    if use_native(qkv):
        ops = native()
        q = ops.rope_append(qkv.contiguous(), cos, sin, pos, slots, k_cache, v_cache, Hq, Hkv, D, block_table)
        return ops.decode_attn(q, k_cache, v_cache, pos, slots, max_len, 1.0 / math.sqrt(D), 1, block_table,
                               counters)
    bt = block_table.cpu() if block_table is not None else None
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
        _kv_at(k_cache, bt, s, p, p + 1)[:, 0] = ki.to(k_cache.dtype)
        _kv_at(v_cache, bt, s, p, p + 1)[:, 0] = x[i, Hq + Hkv:].to(v_cache.dtype)
        kk = _kv_at(k_cache, bt, s, 0, p + 1).float().repeat_interleave(Hq // Hkv, 0)  # [Hq, L, D]
        vv = _kv_at(v_cache, bt, s, 0, p + 1).float().repeat_interleave(Hq // Hkv, 0)
        sc = torch.einsum("hd,hld->hl", qi, kk) / math.sqrt(D)
        outs.append(torch.einsum("hl,hld->hd", sc.softmax(-1), vv).reshape(-1))
    return torch.stack(outs).to(qkv.dtype)


def sample(logits: torch.Tensor, temperature: float = 0.0, seed: int = 0, step: int = 0,
           top_p: float = 1.0, top_k: int = 0) -> torch.Tensor:
    """logits [B, V] -> token ids [B] int64, every row with the same parameters
    (see ``sample_rows``)."""
    B = logits.shape[0]
    return sample_rows(logits, [temperature] * B, [top_p] * B, [top_k] * B, [seed] * B, [step] * B)


def sample_rows(logits: torch.Tensor, temps, top_ps, top_ks, seeds, steps) -> torch.Tensor:
    """Batched sampling with per-row parameters (OpenAI semantics): softmax of
    logits / T, keep the top_k most likely (k <= 0: all), then the smallest
    most-likely prefix whose mass reaches top_p, renormalise, draw; T <= 0 is
    greedy.  GPU: ONE launch for the whole batch (csrc/kernels/sampling.hip:
    radix-select thresholds + Gumbel-max over the kept set, keyed by
    (seed, step, token) so a request's draws do not depend on batching).
    CPU: ``filter_probs`` + torch.multinomial.  ``top_p <= 0`` (an empty nucleus)
    is the limit of a vanishing nucleus: that row is sampled greedily on both paths;
    a NaN top_p / temperature is rejected."""
    B = logits.shape[0]
    temps, top_ps = list(temps), list(top_ps)
    for i, (t, p) in enumerate(zip(temps, top_ps)):
        if p != p or t != t:
            raise ValueError(f"row {i}: top_p={p}, temperature={t} (NaN)")
        if p <= 0:
            temps[i], top_ps[i] = 0.0, 1.0
    if use_native(logits):
        ops = native()
        x = logits if logits.dtype in (torch.bfloat16, torch.float32) else logits.float()
        x = x.contiguous()
        if all(t <= 0 for t in temps):
            return ops.sample(x, 0.0, 0, 0)  # batched greedy: one argmax pass
        dev = logits.device
        prm = torch.tensor([[float(t), float(p), float(k)] for t, p, k in zip(temps, top_ps, top_ks)],
                           dtype=torch.float32).pin_memory().to(dev, non_blocking=True)
        st = torch.tensor([[int(sd), int(sp)] for sd, sp in zip(seeds, steps)], dtype=torch.int64).pin_memory()
        st = st.to(dev, non_blocking=True)
        if all(p >= 1.0 for p in top_ps) and all(k <= 0 for k in top_ks):
            # temperature / greedy rows only: the vocabulary-split kernel (same draws)
            return ops.sample_temp_rows(x, prm[:, 0].contiguous(), st[:, 0].contiguous(), st[:, 1].int().contiguous())
        return ops.sample_rows(x, prm[:, 0].contiguous(), prm[:, 1].contiguous(), prm[:, 2].int().contiguous(),
                               st[:, 0].contiguous(), st[:, 1].int().contiguous())
    out = torch.empty(B, dtype=torch.long)
    for i in range(B):
        if temps[i] <= 0:
            out[i] = logits[i].float().argmax()
            continue
        g = torch.Generator(device=logits.device)
        g.manual_seed(int(seeds[i]) * 1000003 + int(steps[i]))
        pr = filter_probs(logits[i], temps[i], top_ks[i], top_ps[i])
        out[i] = torch.multinomial(pr, 1, generator=g)[0]
    return out.to(logits.device)


def filter_probs(row: torch.Tensor, temperature: float, top_k: int = 0, top_p: float = 1.0) -> torch.Tensor:
    """fp32 reference of the sampling distribution of one logits row: softmax(row / T)
    restricted to the top_k most likely tokens, then to the smallest most-likely
    prefix reaching top_p of that mass (the crossing token kept), renormalised.
    Ties at a boundary are kept (the GPU kernel's threshold semantics)."""
    x = row.float() / max(float(temperature), 1e-20)
    keep = torch.ones_like(x, dtype=torch.bool)
    if 0 < top_k < x.numel():
        kth = torch.topk(x, top_k).values[-1]
        keep &= x >= kth
    p = torch.softmax(x.masked_fill(~keep, float("-inf")), -1)
    if top_p < 1.0:
        srt, idx = torch.sort(p, descending=True)
        before = srt.cumsum(0) - srt  # mass strictly above each token
        cut = srt[(before < top_p * srt.sum()).nonzero().max()]  # smallest kept probability
        keep &= p >= cut
        p = torch.softmax(x.masked_fill(~keep, float("-inf")), -1)
    return p
