"""Tensor parallelism for serving (Megatron-style head / FFN sharding over xGMI).

The reference reaches its Llama-3.1-70B only through a remote endpoint
(reference src/distributed_inference.py:34-41); mxllm serves
it locally.  One MI355X holds the whole bf16 70B (141 GB of 288 GB), so data
parallel replicas are the throughput default, but a single request's decode
latency is bound by streaming every weight once per token (~29 ms bf16 on one
GPU).  Tensor parallelism splits that stream over the node's GPUs:

  * Wqkv is column-parallel by attention head: rank r keeps q heads
    [r*Hq/tp, (r+1)*Hq/tp) and kv heads [r*Hkv/tp, ...) (GQA groups never
    straddle ranks), so RoPE, the KV cache and both attention kernels run on
    local heads with no communication;
  * Wo is row-parallel (input columns of the local heads): partial sums, one
    all-reduce of [tokens, hidden];
  * Wgate/Wup are column-parallel over the FFN dimension, Wdown row-parallel:
    SwiGLU stays local, one all-reduce;
  * the LM head is vocab-parallel (rows padded to a common shard size), the
    logits are all-gathered so every rank samples the same token from the same
    bitwise logits (no broadcast of the choice needed);
  * embedding and RMSNorm weights are replicated (a row gather and a
    [hidden] vector).

Per token and layer this is two all-reduces of ``tokens x hidden`` bf16 — at
decode that is 16 KB per sequence for 70B, a latency-bound message.  On one
8-GPU node those go through a graph-safe one-shot xGMI kernel
(``XgmiGraphComm``: every rank pushes its partial straight into all 7 peers'
buffers over the direct links and reduces locally in rank order; epochs live
in device memory so the launch is captured into the engine's decode hipGraph
with the rest of the step); prefill-sized reductions and the logits gather
use RCCL (``torch.distributed`` "nccl" backend, also graph-captured).  Divisibility: tp must
divide n_kv_heads (8 for Llama-3.1 8B/70B -> tp in {1, 2, 4, 8}) and ffn.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.config import LlamaConfig


def shard_config(cfg: LlamaConfig, tp: int) -> LlamaConfig:
    """Per-rank architecture: local heads / FFN width, same hidden and vocab."""
    if tp < 1 or cfg.n_kv_heads % tp or cfg.n_heads % tp or cfg.ffn % tp:
        raise ValueError(f"tensor-parallel degree {tp} must divide n_kv_heads={cfg.n_kv_heads}, "
                         f"n_heads={cfg.n_heads} and ffn={cfg.ffn}")
    return cfg.replace(n_heads=cfg.n_heads // tp, n_kv_heads=cfg.n_kv_heads // tp, ffn=cfg.ffn // tp,
                       tie_embeddings=False)


def vocab_shard_rows(vocab: int, tp: int) -> int:
    """Rows of each rank's LM-head shard (padded to a multiple of 64)."""
    return int(math.ceil(vocab / tp / 64.0)) * 64


@torch.no_grad()
def shard_llama(full, rank: int, tp: int, device=None):
    """Rank ``rank``'s tensor-parallel shard of a (LoRA-merged) ``Llama``."""
    from ..models.llama import Llama

    cfg = full.cfg
    if any(getattr(m, "lora_r", 0) for m in full.modules()):
        raise ValueError("merge LoRA adapters first (mxllm.serve.engine.merge_lora_)")
    lc = shard_config(cfg, tp)
    device = torch.device(device) if device is not None else full.tok_emb.device
    dt = full.tok_emb.dtype
    local = Llama(lc, device=device, dtype=dt, init=False)
    local.tok_emb.copy_(full.tok_emb)
    local.final_norm.copy_(full.final_norm)
    qd, kd, f = lc.q_dim, lc.kv_dim, lc.ffn
    for src, dst in zip(full.layers, local.layers):
        dst.attn_norm.copy_(src.attn_norm)
        dst.mlp_norm.copy_(src.mlp_norm)
        w = src.wqkv.weight
        q0, k0, v0 = rank * qd, cfg.q_dim + rank * kd, cfg.q_dim + cfg.kv_dim + rank * kd
        dst.wqkv.weight.copy_(torch.cat([w[q0:q0 + qd], w[k0:k0 + kd], w[v0:v0 + kd]], 0))
        dst.wo.weight.copy_(src.wo.weight[:, rank * qd:(rank + 1) * qd])
        w = src.wgu.weight
        dst.wgu.weight.copy_(torch.cat([w[rank * f:(rank + 1) * f], w[cfg.ffn + rank * f:cfg.ffn + (rank + 1) * f]],
                                       0))
        dst.wd.weight.copy_(src.wd.weight[:, rank * f:(rank + 1) * f])
    local.lm_head = nn.Parameter(_head_shard(full.head_weight, rank, tp).to(device), requires_grad=False)
    local.tp_vocab = cfg.vocab_size
    return local.eval()


def random_shard(cfg: LlamaConfig, rank: int, tp: int, device, seed: int = 0, dtype=torch.bfloat16):
    """A random-init rank shard with the exact per-rank shapes of ``cfg`` at
    degree ``tp`` (benchmarks: no rank ever materialises the full model)."""
    from ..models.llama import Llama

    lc = shard_config(cfg, tp)
    local = Llama(lc, device=device, dtype=dtype, seed=seed + 7919 * rank, init=True)
    # replicated pieces must agree across ranks
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    with torch.no_grad():
        local.tok_emb.normal_(0.0, 0.02, generator=gen)
        head = torch.empty(vocab_shard_rows(cfg.vocab_size, tp), cfg.hidden, dtype=dtype, device=device)
        head.normal_(0.0, 0.02, generator=gen)
    local.lm_head = nn.Parameter(head, requires_grad=False)
    local.tp_vocab = cfg.vocab_size
    for p in local.parameters():
        p.requires_grad_(False)
    return local.eval()


def _head_shard(w: torch.Tensor, rank: int, tp: int) -> torch.Tensor:
    V, H = w.shape
    rows = vocab_shard_rows(V, tp)
    out = torch.zeros(rows, H, dtype=w.dtype, device=w.device)
    lo, hi = rank * rows, min((rank + 1) * rows, V)
    if hi > lo:
        out[:hi - lo].copy_(w[lo:hi])
    return out


class TPComm:
    """The two collectives of a tensor-parallel forward over ``group``.

    Partial-sum all-reduces up to ``max_xgmi_elems`` bf16 elements (decode
    batches: B x hidden) go through the graph-safe xGMI one-shot kernel when
    every rank of the group is on this node (``mxllm/parallel/xgmi.py``
    ``XgmiGraphComm``: each rank pushes its partial into all peers' buffers
    over the direct links, one hop, no RCCL channel setup); larger ones
    (prefill) and non-GPU groups use ``torch.distributed`` (RCCL / gloo).
    The choice depends only on the tensor size, so every rank takes the same
    path for the same call."""

    def __init__(self, group, vocab: int, device=None, max_xgmi_elems: int = 1 << 19):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.vocab = vocab
        self.xgmi = None
        if (device is not None and device.type == "cuda" and self.world > 1
                and os.environ.get("MXLLM_TP_XGMI", "1") != "0"):
            from . import xgmi

            self.xgmi = xgmi.create(device, group, cls=xgmi.XgmiGraphComm, max_elems=max_xgmi_elems)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.xgmi is not None and self.xgmi.fits(t):
            return self.xgmi.all_reduce_(t)
        dist.all_reduce(t, group=self.group)
        return t

    def close(self):
        if self.xgmi is not None:
            self.xgmi.close()
            self.xgmi = None

    def gather_logits(self, local: torch.Tensor) -> torch.Tensor:
        """[B, V_shard] per rank -> [B, vocab] (identical on every rank)."""
        B, Vl = local.shape
        local = local.contiguous()
        if dist.get_backend(self.group) == "gloo":
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local, group=self.group)
            return torch.cat(parts, 1)[:, :self.vocab]
        buf = torch.empty(self.world * B, Vl, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(buf, local, group=self.group)
        return buf.view(self.world, B, Vl).permute(1, 0, 2).reshape(B, self.world * Vl)[:, :self.vocab]
