"""Sequence parallelism: Ulysses-style all-to-all head resharding.

Long-context fine-tuning on the 8-GPU xGMI mesh: each rank of a sequence-
parallel (SP) group holds S/P consecutive tokens of every sequence.  Every
token-local op (embedding, RMSNorm, projections, SwiGLU, LoRA, fused CE) runs
on the local shard unchanged; only attention needs the whole sequence, so
around it the activations are re-sharded by heads with one all-to-all each
way (``all_to_all_single`` = RCCL all-to-all, every rank talking to every
peer over its own xGMI link at once — the pattern the fully connected mesh is
built for):

    qkv [B, S/P, (Hq+2Hkv) D]  --a2a-->  [B, S, (Hq+2Hkv)/P D]   (heads of this rank)
    attention (HIP flash kernel, RoPE at global positions 0..S-1)
    o   [B, S, Hq/P D]        --a2a-->  [B, S/P, Hq D]

Requires Hkv % P == 0 (Llama-3.1: 8 KV heads -> P in {1, 2, 4, 8}).  The
all-to-all is its own adjoint, so the backward is the same exchange on the
gradients.  Gradients of replicated parameters are averaged over the whole
world by DDP: each rank's loss is the mean over its local tokens, so the
world average is the full-sequence mean (equal token counts per shard).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import ops


class _AllToAll(torch.autograd.Function):
    """Equal-split all_to_all_single along dim 0 (chunk j -> rank j)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        x = x.contiguous()
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty_like(g)
        dist.all_to_all_single(out, g, group=ctx.group)
        return out, None


class UlyssesAttention:
    """Callable replacing ``ops.attention_block`` inside a sequence-parallel model."""

    def __init__(self, group=None):
        self.group = group
        self.P = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def __call__(self, qkv, cos, sin, B: int, S_local: int, Hq: int, Hkv: int, D: int, causal: bool = True):
        P = self.P
        if Hkv % P or Hq % P:
            raise ValueError(f"sequence parallel degree {P} must divide the head counts ({Hq} q, {Hkv} kv)")
        nq, nk = Hq // P, Hkv // P
        nh = nq + 2 * nk
        x = qkv.view(B, S_local, Hq + 2 * Hkv, D)
        q = x[:, :, :Hq].reshape(B, S_local, P, nq, D)
        k = x[:, :, Hq:Hq + Hkv].reshape(B, S_local, P, nk, D)
        v = x[:, :, Hq + Hkv:].reshape(B, S_local, P, nk, D)
        send = torch.cat([q, k, v], dim=3).permute(2, 0, 1, 3, 4)          # [P(dst head group), B, S/P, nh, D]
        recv = _AllToAll.apply(send, self.group)                            # [P(src seq chunk), B, S/P, nh, D]
        full = recv.permute(1, 0, 2, 3, 4).reshape(B * P * S_local, nh * D)  # [B*S, nh*D], sequence order
        o = ops.attention_block(full, cos, sin, B, P * S_local, nq, nk, D, causal=causal)
        o = o.view(B, P, S_local, nq, D).permute(1, 0, 2, 3, 4)             # [P(dst seq chunk), B, S/P, nq, D]
        back = _AllToAll.apply(o, self.group)                               # [P(src head group), B, S/P, nq, D]
        return back.permute(1, 2, 0, 3, 4).reshape(B * S_local, Hq * D)


def shard_sequence(t: torch.Tensor, group=None) -> torch.Tensor:
    """[B, S] -> this rank's contiguous [B, S/P] slice."""
    P, r = dist.get_world_size(group), dist.get_rank(group)
    S = t.shape[1]
    if S % P:
        raise ValueError(f"sequence length {S} is not divisible by the sequence-parallel degree {P}")
    n = S // P
    return t[:, r * n:(r + 1) * n].contiguous()


def new_groups(sp: int):
    """Partition the world into consecutive-rank SP groups of size ``sp``
    (collective: every rank calls it).  Returns (my SP group, dp_rank, dp_world)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % sp:
        raise ValueError(f"world size {world} is not divisible by sequence-parallel degree {sp}")
    mine = None
    for g in range(world // sp):
        ranks = list(range(g * sp, (g + 1) * sp))
        grp = dist.new_group(ranks)
        if rank in ranks:
            mine = grp
    return mine, rank // sp, world // sp
