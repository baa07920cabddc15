"""Context parallelism: ring attention over the xGMI mesh (SURVEY §5.7 stretch).

Each rank of a context-parallel (CP) group of P ranks holds 2 of the 2P equal
chunks of every sequence in the zigzag layout — chunks r and 2P-1-r — so that
under the causal mask every rank does the same attention work.  Every
token-local op runs on the local tokens unchanged; attention exchanges K/V:
the (K, V) block of the local tokens travels around the ring (P2P
send/recv on RCCL to the next rank, receive from the previous one, issued
before the current block's compute so the transfer hides under it) and each
rank attends its queries to every block it holds, merging the partial outputs
with their log-sum-exps:

    step 0 (own block)        causal attention over the local [chunk r; chunk 2P-1-r]
    block of a rank s < r     all local queries x chunk s           (fully visible)
    block of a rank s > r     queries of chunk 2P-1-r x both chunks  (fully visible)

so each step is ONE call of the HIP flash-attention kernel
(csrc/kernels/attn_fwd.hip) with the usual (O, LSE) outputs.  The backward
re-runs the ring with the final O and the merged LSE: per block the HIP
backward (attn_bwd.hip) gives dQ (accumulated locally) and per-q-head dK/dV
partials, which are summed over the GQA group into f32 dK/dV accumulators
that travel WITH the block and return to their owner after the last step.
RoPE is applied at the tokens' global positions (zigzag positions), and the
inverse-RoPE/GQA merge kernel (rope.hip) produces d(qkv).

Unlike Ulysses (mxllm/parallel/sequence.py) it needs no head divisibility and
its messages are point-to-point (one xGMI link per step), so it scales the
sequence past what one GPU's activations hold.  Reference parity: none — the
reference never tokenises text.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from ..ops import reference as ref
from ..ops._ext import native, use_native


def zigzag_positions(S_local: int, P: int, r: int, device=None) -> torch.Tensor:
    """Global token positions held by rank r: chunk r then chunk 2P-1-r (C = S_local/2)."""
    C = S_local // 2
    a = torch.arange(r * C, (r + 1) * C, device=device)
    b = torch.arange((2 * P - 1 - r) * C, (2 * P - r) * C, device=device)
    return torch.cat([a, b])


def zigzag_shard(t: torch.Tensor, group=None) -> torch.Tensor:
    """[B, S, ...] -> this rank's zigzag [B, S/P, ...] (chunks r and 2P-1-r of 2P)."""
    P, r = dist.get_world_size(group), dist.get_rank(group)
    S = t.shape[1]
    if S % (2 * P):
        raise ValueError(f"sequence length {S} is not divisible by 2 x context-parallel degree {P}")
    C = S // (2 * P)
    return torch.cat([t[:, r * C:(r + 1) * C], t[:, (2 * P - 1 - r) * C:(2 * P - r) * C]], dim=1).contiguous()


def zigzag_unshard(parts: list[torch.Tensor]) -> torch.Tensor:
    """Inverse of zigzag_shard given every rank's [B, S/P, ...] part (tests)."""
    P = len(parts)
    C = parts[0].shape[1] // 2
    chunks = [None] * (2 * P)
    for r, p in enumerate(parts):
        chunks[r], chunks[2 * P - 1 - r] = p[:, :C], p[:, C:]
    return torch.cat(chunks, dim=1)


# --------------------------------------------------------------------- per-block primitives
def _blk_fwd(q, k, v, causal: bool, scale: float):
    """q [B,Hq,Sq,D], k/v [B,Hkv,Sk,D] -> (o token-major [B,Sq,Hq*D], lse [B,Hq,Sq] log2 domain)."""
    if use_native(q):
        return native().attn_fwd(q.contiguous(), k.contiguous(), v.contiguous(), causal, scale)
    B, Hq, Sq, D = q.shape
    rep = Hq // k.shape[1]
    kf = k.float().repeat_interleave(rep, 1)
    vf = v.float().repeat_interleave(rep, 1)
    s = torch.matmul(q.float(), kf.transpose(-1, -2)) * scale
    if causal:
        Sk = k.shape[2]
        i = torch.arange(Sq).view(Sq, 1)
        j = torch.arange(Sk).view(1, Sk)
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.matmul(torch.exp(s - lse.unsqueeze(-1)), vf)
    return o.transpose(1, 2).reshape(B, Sq, Hq * D).to(q.dtype), lse / math.log(2.0)


def _blk_bwd(do, q, k, v, o, lse, causal: bool, scale: float):
    """Gradients of one block given the FINAL o and merged lse (log2):
    dq f32 [B,Hq,Sq,D], per-q-head dk/dv partials f32 [B,Hq,Sk,D]."""
    if use_native(q):
        return native().attn_bwd(do.contiguous(), q.contiguous(), k.contiguous(), v.contiguous(), o.contiguous(),
                                 lse.contiguous(), causal, scale)
    B, Hq, Sq, D = q.shape
    Sk = k.shape[2]
    rep = Hq // k.shape[1]
    qf, kf, vf = q.float(), k.float().repeat_interleave(rep, 1), v.float().repeat_interleave(rep, 1)
    dof = do.float().view(B, Sq, Hq, D).transpose(1, 2)
    of = o.float().view(B, Sq, Hq, D).transpose(1, 2)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    p = torch.exp(s - (lse * math.log(2.0)).unsqueeze(-1))
    if causal:
        i = torch.arange(Sq).view(Sq, 1)
        j = torch.arange(Sk).view(1, Sk)
        p = p.masked_fill(j > i + (Sk - Sq), 0.0)
    delta = (dof * of).sum(-1, keepdim=True)
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dpv = torch.matmul(dof, vf.transpose(-1, -2))
    ds = p * (dpv - delta)
    dq = torch.matmul(ds, kf) * scale
    dk = torch.matmul(ds.transpose(-1, -2), qf) * scale
    return dq, dk, dv


def _merge(o_acc, lse_acc, o_i, lse_i, rows=None):
    """In-place online merge of a partial (o_i token-major, lse_i log2) into the
    f32 accumulators; ``rows`` = slice of the accumulator rows it covers."""
    B, Sa, HD = o_acc.shape
    Hq = lse_acc.shape[1]
    sl = slice(None) if rows is None else rows
    la = lse_acc[:, :, sl]
    new = torch.logaddexp2(la, lse_i)
    wa = torch.exp2(la - new).transpose(1, 2).unsqueeze(-1)  # [B, S, Hq, 1]
    wi = torch.exp2(lse_i - new).transpose(1, 2).unsqueeze(-1)
    oa = o_acc[:, sl].view(B, -1, Hq, HD // Hq)
    oa.mul_(wa).add_(o_i.float().view(B, -1, Hq, HD // Hq) * wi)
    lse_acc[:, :, sl] = new


class _Ring:
    """K/V (and in backward, dK/dV) blocks passed to the next rank of the group."""

    def __init__(self, group):
        self.group = group
        self.P = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.P))
        self.nxt, self.prv = ranks[(self.r + 1) % self.P], ranks[(self.r - 1) % self.P]

    def start(self, send: torch.Tensor):
        recv = torch.empty_like(send)
        ops = [dist.P2POp(dist.isend, send, self.nxt, self.group), dist.P2POp(dist.irecv, recv, self.prv, self.group)]
        return recv, dist.batch_isend_irecv(ops)

    @staticmethod
    def wait(works):
        for w in works:
            w.wait()


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos_l, sin_l, ring, B, S, Hq, Hkv, D):
        P, r = ring.P, ring.r
        scale = 1.0 / math.sqrt(D)
        if use_native(qkv):
            q, k, v = native().rope_split(qkv.contiguous(), cos_l, sin_l, B, S, Hq, Hkv, D, None)
        else:
            x = qkv.view(B, S, Hq + 2 * Hkv, D)
            q = ref.apply_rope(x[:, :, :Hq], cos_l, sin_l).transpose(1, 2).contiguous()
            k = ref.apply_rope(x[:, :, Hq:Hq + Hkv], cos_l, sin_l).transpose(1, 2).contiguous()
            v = x[:, :, Hq + Hkv:].transpose(1, 2).contiguous()
        C = S // 2
        kv = torch.stack([k, v])  # [2, B, Hkv, S, D]: the block that travels
        o_acc = torch.zeros(B, S, Hq * D, dtype=torch.float32, device=qkv.device)
        lse_acc = torch.full((B, Hq, S), float("-inf"), dtype=torch.float32, device=qkv.device)
        cur = kv
        for step in range(P):
            pending = ring.start(cur) if step + 1 < P else None  # next block in flight under this compute
            s = (r - step) % P
            kb, vb = cur[0], cur[1]
            if s == r:
                o_i, l_i = _blk_fwd(q, kb, vb, True, scale)
                _merge(o_acc, lse_acc, o_i, l_i)
            elif s < r:
                o_i, l_i = _blk_fwd(q, kb[:, :, :C], vb[:, :, :C], False, scale)
                _merge(o_acc, lse_acc, o_i, l_i)
            else:
                o_i, l_i = _blk_fwd(q[:, :, C:], kb, vb, False, scale)
                _merge(o_acc, lse_acc, o_i, l_i, rows=slice(C, S))
            if pending is not None:
                cur, works = pending
                _Ring.wait(works)
        o = o_acc.to(qkv.dtype)
        ctx.save_for_backward(q, k, v, o, lse_acc, cos_l, sin_l)
        ctx.ring, ctx.dims = ring, (B, S, Hq, Hkv, D)
        return o.view(B * S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cos_l, sin_l = ctx.saved_tensors
        ring = ctx.ring
        B, S, Hq, Hkv, D = ctx.dims
        P, r = ring.P, ring.r
        rep = Hq // Hkv
        C = S // 2
        scale = 1.0 / math.sqrt(D)
        do = do.reshape(B, S, Hq * D).contiguous()
        dq = torch.zeros(B, Hq, S, D, dtype=torch.float32, device=q.device)
        kv = torch.stack([k, v])
        dkv = torch.zeros(2, B, Hkv, S, D, dtype=torch.float32, device=q.device)  # travels with kv

        def gsum(t):  # dK / dV partials (per q-head, or per group of q-heads) -> per-kv-head sums
            return t.view(B, Hkv, -1, t.shape[2], D).sum(2)

        cur, dcur = kv, dkv
        for step in range(P):
            pending = ring.start(cur) if step + 1 < P else None
            s = (r - step) % P
            kb, vb = cur[0], cur[1]
            if s == r:
                dq_i, dk_i, dv_i = _blk_bwd(do, q, kb, vb, o, lse, True, scale)
                dq += dq_i
                dcur[0] += gsum(dk_i)
                dcur[1] += gsum(dv_i)
            elif s < r:
                dq_i, dk_i, dv_i = _blk_bwd(do, q, kb[:, :, :C], vb[:, :, :C], o, lse, False, scale)
                dq += dq_i
                dcur[0][:, :, :C] += gsum(dk_i)
                dcur[1][:, :, :C] += gsum(dv_i)
            else:
                dq_i, dk_i, dv_i = _blk_bwd(do[:, C:], q[:, :, C:], kb, vb, o[:, C:], lse[:, :, C:], False, scale)
                dq[:, :, C:] += dq_i
                dcur[0] += gsum(dk_i)
                dcur[1] += gsum(dv_i)
            # the accumulated dK/dV of this block move on with it (after the last step: to its owner)
            dpend = ring.start(dcur) if P > 1 else None
            if pending is not None:
                cur, works = pending
                _Ring.wait(works)
            if dpend is not None:
                dcur, dworks = dpend
                _Ring.wait(dworks)
        dk, dv = dcur[0], dcur[1]  # this rank's own block, complete
        if use_native(q):
            # already one sum per KV head: the merge takes them as Hkv "partials"
            dqkv = native().rope_merge_bwd(dq, dk.contiguous(), dv.contiguous(), cos_l, sin_l, B, S, Hq, Hkv, D, 0)
        else:
            dqr = ref.apply_rope(dq.transpose(1, 2), cos_l, -sin_l)
            dkr = ref.apply_rope(dk.transpose(1, 2), cos_l, -sin_l)
            dqkv = torch.cat([dqr, dkr, dv.transpose(1, 2)], dim=2).reshape(B * S, (Hq + 2 * Hkv) * D)
        return dqkv.to(q.dtype), None, None, None, None, None, None, None, None


class RingAttention:
    """Callable replacing ``ops.attention_block`` inside a context-parallel model
    (same call signature as UlyssesAttention); inputs are this rank's zigzag tokens."""

    def __init__(self, group=None):
        self.group = group
        self.ring = _Ring(group)
        self.P, self.rank = self.ring.P, self.ring.r
        self._pos = {}

    def __call__(self, qkv, cos, sin, B: int, S_local: int, Hq: int, Hkv: int, D: int, causal: bool = True):
        if not causal:
            raise ValueError("ring attention here implements the causal (decoder) case")
        if S_local % 2:
            raise ValueError("zigzag context parallelism needs an even local length")
        key = (S_local, cos.device)
        if key not in self._pos:
            pos = zigzag_positions(S_local, self.P, self.rank, cos.device)
            self._pos[key] = (cos[pos].contiguous(), sin[pos].contiguous())
        cos_l, sin_l = self._pos[key]
        return _RingAttnFn.apply(qkv, cos_l, sin_l, self.ring, B, S_local, Hq, Hkv, D)
