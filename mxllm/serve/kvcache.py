"""Paged KV cache for the serving engine (VERDICT r2 missing #5).

Per layer, K and V are POOLS of fixed-size blocks ``[blocks, Hkv, block, D]``
(bf16) and every sequence slot maps its token positions to pool blocks through
a block table ``bt [slots, max_blocks]`` (int32, on the device).  Token ``p`` of
slot ``s`` lives in block ``bt[s, p // block]`` at row ``p % block``.  The HIP
decode kernels (csrc/kernels/decode.hip ``kv_row``: RoPE + cache append, the
split-K decode attention, the fused QKV GEMM epilogue) read the table; the block
size is a multiple of the 256-key decode split, so every split streams ONE
contiguous block.

Two modes:
  * static (``pool_tokens=None``): every slot owns ``max_blocks`` blocks for
    life — the memory of the old ``[slots, Hkv, max_seq, D]`` slab;
  * paged (``pool_tokens=N``): a shared pool of ``ceil(N / block)`` blocks; a
    request reserves only ``ceil(min(prompt + max_new_tokens, max_seq) / block)``
    blocks at admission and returns them when it finishes.  The reference
    workload's IMDB reviews are ~0.3-4k tokens, so with a 70B model (320 KiB of
    KV per token) a pool sized for the AVERAGE length serves several times more
    concurrent requests than slots sized for the longest one.

One spare slot with one block takes the padding rows of a graphed decode step.
"""
from __future__ import annotations

import math

import torch

BLOCK = 256


class KVCache:
    def __init__(self, n_layers: int, n_kv_heads: int, head_dim: int, dtype, device, n_slots: int, max_seq: int,
                 pool_tokens: int | None = None, block: int = BLOCK, scratch_slot: int | None = None):
        if block % 256:
            raise ValueError("KV block size must be a multiple of 256 tokens (the decode split)")
        self.block = block
        self.max_seq = max_seq
        self.maxb = math.ceil(max_seq / block)
        self.n_slots = n_slots
        self.paged = pool_tokens is not None
        self.scratch_slot = scratch_slot
        if self.paged:
            n_blocks = max(math.ceil(pool_tokens / block), 1)
        else:
            n_blocks = (n_slots - (1 if scratch_slot is not None else 0)) * self.maxb
        n_blocks += 1 if scratch_slot is not None else 0
        self.n_blocks = n_blocks
        self.k = [torch.zeros(n_blocks, n_kv_heads, block, head_dim, dtype=dtype, device=device)
                  for _ in range(n_layers)]
        self.v = [torch.zeros_like(k) for k in self.k]
        self.bt_host = torch.zeros(n_slots, self.maxb, dtype=torch.int32)
        self.owned: dict[int, list[int]] = {}
        self.free: list[int] = []
        if self.paged:
            self.free = list(range(n_blocks - (1 if scratch_slot is not None else 0)))
        else:
            for s in range(n_slots):
                if s == scratch_slot:
                    continue
                j = s - (1 if scratch_slot is not None and s > scratch_slot else 0)
                self.owned[s] = list(range(j * self.maxb, (j + 1) * self.maxb))
                self.bt_host[s] = torch.tensor(self.owned[s], dtype=torch.int32)
        if scratch_slot is not None:
            self.owned[scratch_slot] = [n_blocks - 1]
            self.bt_host[scratch_slot, :] = n_blocks - 1
        self.bt = self.bt_host.to(device)

    # ------------------------------------------------------------------ accounting
    def blocks_for(self, tokens: int) -> int:
        return math.ceil(max(1, min(tokens, self.max_seq)) / self.block)

    @property
    def free_blocks(self) -> int:
        return len(self.free) if self.paged else 0

    def can_reserve(self, tokens: int) -> bool:
        return not self.paged or self.blocks_for(tokens) <= len(self.free)

    def fits_at_all(self, tokens: int) -> bool:
        return not self.paged or self.blocks_for(tokens) <= self.n_blocks - (1 if self.scratch_slot is not None else 0)

    def reserve(self, slot: int, tokens: int) -> None:
        """Give ``slot`` the blocks for positions [0, tokens) (paged mode; a no-op
        in static mode, where every slot owns max_seq positions)."""
        if not self.paged:
            return
        self.release(slot)
        n = self.blocks_for(tokens)
        if n > len(self.free):
            raise RuntimeError(f"KV pool exhausted: need {n} blocks, {len(self.free)} free")
        blocks, self.free = self.free[:n], self.free[n:]
        self.owned[slot] = blocks
        row = torch.zeros(self.maxb, dtype=torch.int32)
        row[:n] = torch.tensor(blocks, dtype=torch.int32)
        row[n:] = blocks[-1]  # never read (lengths stay inside the reservation); keeps the table in range
        self.bt_host[slot] = row
        self.bt[slot].copy_(row.to(self.bt.device), non_blocking=False)

    def capacity(self, slot: int) -> int:
        """Positions ``slot`` can hold."""
        if not self.paged:
            return self.max_seq
        return min(len(self.owned.get(slot, ())) * self.block, self.max_seq)

    def release(self, slot: int) -> None:
        if self.paged and slot in self.owned and slot != self.scratch_slot:
            self.free.extend(self.owned.pop(slot))

    # ------------------------------------------------------------------ data
    def write(self, layer: int, slot: int, k: torch.Tensor, v: torch.Tensor) -> None:
        """Store K/V rows of positions [0, S) of ``slot``: k, v [Hkv, S, D]."""
        Hkv, S, D = k.shape
        nb = math.ceil(S / self.block)
        blocks = self.owned[slot][:nb]
        if len(blocks) < nb:
            raise RuntimeError(f"slot {slot} holds {len(blocks)} KV blocks, {nb} needed")
        kc, vc = self.k[layer], self.v[layer]
        full = S // self.block
        if full and all(blocks[j] == blocks[0] + j for j in range(full)):  # consecutive blocks: views
            b0 = blocks[0]
            kc[b0:b0 + full].copy_(k[:, :full * self.block].view(Hkv, full, self.block, D).transpose(0, 1))
            vc[b0:b0 + full].copy_(v[:, :full * self.block].view(Hkv, full, self.block, D).transpose(0, 1))
        elif full:
            idx = torch.tensor(blocks[:full], device=kc.device)
            kc.index_copy_(0, idx, k[:, :full * self.block].reshape(Hkv, full, self.block, D).transpose(0, 1))
            vc.index_copy_(0, idx, v[:, :full * self.block].reshape(Hkv, full, self.block, D).transpose(0, 1))
        rem = S - full * self.block
        if rem:
            kc[blocks[full], :, :rem].copy_(k[:, full * self.block:])
            vc[blocks[full], :, :rem].copy_(v[:, full * self.block:])

    def gather(self, layer: int, slot: int, L: int) -> tuple[torch.Tensor, torch.Tensor]:
        """K/V of positions [0, L) of ``slot`` as [Hkv, L, D] (reference paths / tests)."""
        nb = math.ceil(L / self.block)
        idx = self.bt_host[slot, :nb].to(torch.long).to(self.k[layer].device)

        def g(c):
            t = c.index_select(0, idx)  # [nb, Hkv, block, D]
            return t.transpose(0, 1).reshape(t.shape[1], nb * self.block, t.shape[3])[:, :L]

        return g(self.k[layer]), g(self.v[layer])

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.k + self.v)
