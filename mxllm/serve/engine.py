"""mxllm inference engine: KV cache + prefill/decode + continuous batching.

This replaces the reference's remote API offload: ``get_model_response``
(reference src/distributed_inference.py:34-41) called an external Llama-3.1-70B
over HTTP, one blocking request per prompt.  Here every rank
serves its own shard of prompts from its own GPU, batched.

MI355X-first sizing: the KV cache (mxllm/serve/kvcache.py) is a pool of
256-token blocks per layer addressed through a per-slot block table.  Static
mode gives every slot max_seq positions (70B: 320 KiB/token, 16 slots x 8k
tokens = 43 GB beside the 141 GB of weights on one 288 GB MI355X); paged mode
(``kv_pool_tokens``) shares a pool and a request reserves only
prompt + max_new_tokens, so many more short requests run at once.  Prefill
runs the MFMA flash-attention kernel; decode runs the split-K decode kernel
(one workgroup streams 256 cached keys of one (sequence, kv-head) and serves
all q-heads of that GQA group).  Scheduling is continuous batching: new
requests are prefilled between decode steps (all prompts admitted together in
one pass: concatenated tokens through the GEMMs, attention per sequence) and
join the running batch.

Decode is launch-bound at small batch (a 32-layer step is ~300 kernel
launches), so on GPU each decode step is replayed from a hipGraph
(``torch.cuda.CUDAGraph`` is hipGraph capture on ROCm).  One graph per
(batch bucket, key-split bucket): the batch is padded to a power of two with
entries that write into a scratch cache slot, the split-K decode kernel gets
a power-of-two key bound (splits past a sequence's length exit at once), and
the step's only host->device traffic is one [3, B] int64 copy of
(token, position, slot).
"""
from __future__ import annotations

import itertools
import logging
import math
import os
import threading
import time
from dataclasses import dataclass, field

import torch

from .. import ops
from ..models.llama import FusedLinear
from ..ops import decode as dops

_SWIGLU_FUSED = os.environ.get("MXLLM_SWIGLU_FUSED", "1") != "0"  # A/B switch (bench/serve_bench.py)
_NORM_FUSED = os.environ.get("MXLLM_NORM_FUSED", "1") != "0"  # A/B switch: RMSNorm in the decode GEMM prologue
_ROPE_FUSED = os.environ.get("MXLLM_ROPE_FUSED", "1") != "0"  # A/B switch: RoPE + cache append in the QKV epilogue
# the split-K attention merge in the o-projection GEMM's prologue (decode rows <= 4): OFF by
# default -- measured 8B decode, same box: batch 1 3.424 vs 3.433 ms (a wash), batch 4 4.113 vs
# 3.841 ms (the prologue slows the weight stream more than the combine launch costs;
# archive/profiles/r3d_decode_merge_ab.md).  MXLLM_MERGE_FUSED=1 turns it on.
_MERGE_FUSED = os.environ.get("MXLLM_MERGE_FUSED", "0") == "1"
# Small-batch decode: while the (latency-bound) attention runs, a side-stream kernel reads
# the layer's o-projection weight so the o-projection GEMM streams it from the Infinity
# Cache instead of HBM (MXLLM_DECODE_PREFETCH=1; up to PREFETCH_MAX_B rows).  Measured
# slower (fork/join + competing reads; archive/profiles/r3g/README.md): off by default.
_PREFETCH = os.environ.get("MXLLM_DECODE_PREFETCH", "0") == "1"
PREFETCH_MAX_B = 8
log = logging.getLogger("mxllm.engine")


@dataclass
class SamplingParams:
    max_new_tokens: int = 64
    temperature: float = 0.0
    top_p: float = 1.0
    top_k: int = 0
    stop_ids: tuple = ()
    seed: int = 0

    def __post_init__(self):
        if not (self.top_p == self.top_p and self.temperature == self.temperature):
            raise ValueError("top_p / temperature must not be NaN")
        if self.top_p < 0:
            raise ValueError(f"top_p must be in [0, 1] (0 = greedy), got {self.top_p}")
        if self.max_new_tokens < 0:
            raise ValueError(f"max_new_tokens must be >= 0, got {self.max_new_tokens}")


@dataclass
class Request:
    rid: int
    prompt: list
    params: SamplingParams
    output: list = field(default_factory=list)
    slot: int = -1
    done: threading.Event = field(default_factory=threading.Event)
    finish_reason: str | None = None
    t_submit: float = field(default_factory=time.perf_counter)
    t_first: float | None = None
    t_done: float | None = None
    error: str | None = None


class Engine:
    def __init__(self, model, max_batch: int = 8, max_seq: int = 4096, device=None, eos_ids=(),
                 use_graphs: bool | None = None, prefill_tokens: int = 16384, tp_group=None,
                 kv_pool_tokens: int | None = None, kv_block: int = 256):
        """``tp_group``: serve a tensor-parallel shard (mxllm/parallel/tensor.py
        ``shard_llama`` / ``random_shard``) with the other ranks of the group;
        every rank of the group runs the same schedule (same submissions in the
        same order, e.g. SPMD ``generate`` or ``serve_follower``).
        ``kv_pool_tokens``: paged KV cache of that many tokens shared by all slots
        (None: every slot owns max_seq positions; env MXLLM_KV_POOL_TOKENS)."""
        self.model = model
        self.tp = None
        if tp_group is not None:
            from ..parallel.tensor import TPComm

            self.tp = TPComm(tp_group, getattr(model, "tp_vocab", model.cfg.vocab_size),
                             device=device or model.tok_emb.device)
            if self.tp.world == 1:
                self.tp = None
        self.prefill_budget = max(1, prefill_tokens)  # tokens per prefill pass
        self.cfg = model.cfg
        self.device = device or model.tok_emb.device
        self.max_batch = max_batch
        self.max_seq = min(max_seq, self.cfg.max_seq_len)
        if self.device.type == "cuda":
            # tuned hipBLASLt/rocBLAS solution table (read-only; incl. the 70B decode shapes,
            # bench/tune_decode_gemms.py); MXLLM_GEMM_TUNING=0 keeps the library defaults
            from ..utils import gemm_tuning

            gemm_tuning.enable()
        if use_graphs is None:
            use_graphs = self.device.type == "cuda" and os.environ.get("MXLLM_DECODE_GRAPHS", "1") != "0"
            if self.tp is not None:  # RCCL collectives are graph-capturable, gloo's are not
                import torch.distributed as dist

                use_graphs = use_graphs and dist.get_backend(self.tp.group) == "nccl"
        self.use_graphs = bool(use_graphs)
        self._graphs: dict = {}
        self._pool = None
        self.scratch_slot = max_batch  # padding rows of a graphed step write here
        c = self.cfg
        dt = model.tok_emb.dtype
        n_slots = max_batch + (1 if self.use_graphs else 0)
        if kv_pool_tokens is None and os.environ.get("MXLLM_KV_POOL_TOKENS"):
            kv_pool_tokens = int(os.environ["MXLLM_KV_POOL_TOKENS"])
        from .kvcache import KVCache

        self.kv = KVCache(c.n_layers, c.n_kv_heads, c.head_dim, dt, self.device, n_slots, self.max_seq,
                          pool_tokens=kv_pool_tokens, block=kv_block,
                          scratch_slot=self.scratch_slot if self.use_graphs else None)
        # MXLLM_DECODE_COMBINE=fused: the split-K partials merge inside the attention launch (the
        # last workgroup of each (seq, kv-head) combines; these counters stay zero between calls)
        # instead of the combine kernel -- measured slower in the graphed step at every batch
        # (archive/profiles/r3g/README.md), so off by default
        self._attn_cnt = None
        if self.device.type == "cuda" and os.environ.get("MXLLM_DECODE_COMBINE", "kernel") == "fused":
            self._attn_cnt = torch.zeros((n_slots + 64) * self.kv.k[0].shape[1], dtype=torch.int32,
                                         device=self.device)
        self._pf_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" and _PREFETCH else None
        self.eos_ids = tuple(eos_ids) if eos_ids else (c.eos_id,)
        self.free_slots = list(range(max_batch))
        self.active: dict[int, Request] = {}
        self.waiting: list[Request] = []
        self.lens = [0] * max_batch
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._thread = None
        self._stop = False
        self._tasks: list = []  # (fn, result box, event): run by the engine thread between steps
        self.steps = 0
        self.tokens_generated = 0
        # latency / throughput counters: exported by the server's
        # /metrics and by stats()
        self.prefill_tokens = 0
        self.prefill_s = 0.0
        self.decode_s = 0.0
        self.decode_tokens = 0
        self.ttft_sum = 0.0
        self.latency_sum = 0.0
        self.finished = 0

    # ------------------------------------------------------------------ model pieces
    def _norm_proj(self, delta, h, gamma, lin, swiglu: bool):
        """(proj(rmsnorm(h + delta) * gamma), h + delta); ``swiglu``: proj = swiglu(lin(.)).
        Decode rows of a plain bf16 projection run as ONE launch (RMSNorm in the GEMM
        prologue, SwiGLU in its epilogue: csrc/kernels/skinny_gemm.hip)."""
        eps = self.cfg.norm_eps
        plain = type(lin) is FusedLinear and lin.lora_r == 0
        if _NORM_FUSED and plain:
            r = ops.norm_linear(delta, h, gamma, eps, lin.weight, swiglu)
            if r is not None:
                return r
        if delta is None:
            xn = ops.rms_norm(h, gamma, eps)
        else:
            xn, h = ops.add_rms_norm(delta, h, gamma, eps)
        if not swiglu:
            return lin(xn), h
        mid = None
        if _SWIGLU_FUSED and plain and xn.dim() == 2:
            mid = ops.linear_swiglu(xn, lin.weight)  # decode rows: SwiGLU in the GEMM epilogue
        if mid is None:
            mid = ops.swiglu(lin(xn))
        return mid, h

    @torch.no_grad()
    def _layers(self, x: torch.Tensor, attn_fn, qkv_fn=None) -> torch.Tensor:
        """``qkv_fn(i, delta, h, gamma, layer)`` (decode): the fused norm + QKV + RoPE/cache-append
        projection returning (rotated q, new residual) or None; ``attn_fn(i, qkv, q=None)``."""
        m, c = self.model, self.cfg
        h = x
        delta, gamma = None, m.layers[0].attn_norm  # sub-block output not yet added to h, next norm
        for i, layer in enumerate(m.layers):
            r = qkv_fn(i, delta, h, gamma, layer) if qkv_fn is not None else None
            if r is not None:
                q, h = r
                o = attn_fn(i, None, q)
            else:
                qkv, h = self._norm_proj(delta, h, gamma, layer.wqkv, False)
                o = attn_fn(i, qkv)
            if isinstance(o, tuple):  # split-K partials: merged in the o-projection's prologue
                a = ops.native().skinny_merge_linear(o[0], o[1], layer.wo.weight)
            else:
                a = layer.wo(o)
            if self.tp is not None:  # row-parallel Wo: sum the heads' partial outputs
                self.tp.all_reduce_(a)
            mid, h = self._norm_proj(a, h, layer.mlp_norm, layer.wgu, True)
            d = layer.wd(mid)
            if self.tp is not None:  # row-parallel Wdown
                self.tp.all_reduce_(d)
            delta, gamma = d, (m.layers[i + 1].attn_norm if i + 1 < len(m.layers) else m.final_norm)
        if delta is None:
            return ops.rms_norm(h, gamma, c.norm_eps)
        xn, h = ops.add_rms_norm(delta, h, gamma, c.norm_eps)
        return xn

    @property
    def k_cache(self):
        return self.kv.k

    @property
    def v_cache(self):
        return self.kv.v

    def reserve(self, slot: int, tokens: int) -> None:
        """Make ``slot`` able to hold ``tokens`` positions (paged KV: take blocks from the
        pool; static: nothing to do).  The scheduler reserves prompt + max_new_tokens at
        admission; direct ``prefill`` / ``decode`` callers may reserve themselves."""
        self.kv.reserve(slot, tokens)

    def _ensure(self, slot: int, tokens: int) -> None:
        if self.kv.capacity(slot) < tokens:
            if self.kv.paged and not self.kv.owned.get(slot):
                self.kv.reserve(slot, self.max_seq if self.kv.can_reserve(self.max_seq) else tokens)
            else:
                raise ValueError(f"slot {slot} holds {self.kv.capacity(slot)} KV positions, {tokens} needed")

    @torch.no_grad()
    def prefill(self, slot: int, ids: list[int]) -> torch.Tensor:
        """Run the prompt through the model, filling ``slot``'s cache; returns
        last-position logits [V] (f32)."""
        m, c = self.model, self.cfg
        S = len(ids)
        if S >= self.max_seq:
            raise ValueError(f"prompt of {S} tokens exceeds max_seq {self.max_seq}")
        self._ensure(slot, S + 1)
        t = torch.tensor(ids, dtype=torch.long, device=self.device)
        x = ops.embedding(t, m.tok_emb)

        def attn(i, qkv):
            return dops.prefill_attention(qkv, m.rope_cos, m.rope_sin, lambda k, v: self.kv.write(i, slot, k, v),
                                          S, c.n_heads, c.n_kv_heads, c.head_dim)

        xn = self._layers(x, attn)
        self.lens[slot] = S
        return self._logits(xn[-1:]).float()[0]

    def _logits(self, xn: torch.Tensor) -> torch.Tensor:
        out = ops.linear(xn, self.model.head_weight)  # decode rows: the weight-streaming HIP GEMM
        if self.tp is not None:  # vocab-parallel head
            out = self.tp.gather_logits(out)
        return out

    @torch.no_grad()
    def prefill_batch(self, slots: list[int], prompts: list[list[int]]) -> torch.Tensor:
        """Prefill several prompts in ONE pass: their tokens are concatenated so
        every GEMM / norm / SwiGLU runs once over all of them (each weight is
        read once per batch instead of once per prompt); attention runs per
        sequence into its own cache slot.  Returns last-position logits [n, V] f32."""
        m, c = self.model, self.cfg
        lens = [len(p) for p in prompts]
        if any(S >= self.max_seq for S in lens):
            raise ValueError(f"prompt exceeds max_seq {self.max_seq}")
        for s_, S in zip(slots, lens):
            self._ensure(s_, S + 1)
        t = torch.tensor([tok for p in prompts for tok in p], dtype=torch.long, device=self.device)
        x = ops.embedding(t, m.tok_emb)
        offs = [0]
        for S in lens:
            offs.append(offs[-1] + S)

        def attn(i, qkv):
            outs = [dops.prefill_attention(qkv[offs[j]:offs[j + 1]], m.rope_cos, m.rope_sin,
                                           lambda k, v, j=j: self.kv.write(i, slots[j], k, v), lens[j], c.n_heads,
                                           c.n_kv_heads, c.head_dim)
                    for j in range(len(prompts))]
            return outs[0] if len(outs) == 1 else torch.cat(outs, 0)

        xn = self._layers(x, attn)
        for s_, S in zip(slots, lens):
            self.lens[s_] = S
        last = torch.tensor([o - 1 for o in offs[1:]], device=self.device)
        return self._logits(xn.index_select(0, last)).float()

    @torch.no_grad()
    def decode(self, slots: list[int], tokens: torch.Tensor) -> torch.Tensor:
        """One token for each sequence in ``slots``; returns logits [B, V]."""
        B = len(slots)
        max_len = max(self.lens[s] for s in slots) + 1
        for s in slots:
            self._ensure(s, self.lens[s] + 1)
        if self.use_graphs:
            logits = self._decode_graphed(slots, tokens, max_len)
        else:
            inp = torch.stack([tokens.to(self.device, torch.long),
                               torch.tensor([self.lens[s] for s in slots], device=self.device),
                               torch.tensor(slots, device=self.device)])
            logits = self._decode_body(inp, max_len)
        for s in slots:
            self.lens[s] += 1
        return logits[:B]

    def _decode_body(self, inp: torch.Tensor, max_len: int) -> torch.Tensor:
        """inp int64 [3, B] = (token, position of the new token, cache slot)."""
        m, c = self.model, self.cfg
        pos = inp[1].to(torch.int32)
        sl = inp[2].to(torch.int32)
        x = ops.embedding(inp[0], m.tok_emb)

        bt = self.kv.bt
        B = inp.shape[1]
        nsplit = (min(max_len, self.kv.maxb * self.kv.block) + 255) // 256
        merge = _MERGE_FUSED and c.head_dim == 128 and B <= 4 and nsplit <= 16
        cnt = self._attn_cnt
        if cnt is not None and B * self.kv.k[0].shape[1] > cnt.numel():
            cnt = None

        pf = self._pf_stream if B <= PREFETCH_MAX_B else None

        def attn(i, qkv, q=None):
            if pf is None:
                return attn_(i, qkv, q)
            wo = getattr(m.layers[i].wo, "weight", None)
            if wo is None or not wo.is_contiguous():
                return attn_(i, qkv, q)
            cur = torch.cuda.current_stream(self.device)
            pf.wait_stream(cur)
            with torch.cuda.stream(pf):
                ops.native().prefetch(wo, 128)
            out = attn_(i, qkv, q)
            cur.wait_stream(pf)  # joins the side branch before the o-projection
            return out

        def attn_(i, qkv, q=None):
            if q is not None:  # RoPE and the cache append already done by the QKV GEMM
                wo = m.layers[i].wo
                K = q.shape[1] * 128  # this rank's heads (tensor parallel: a shard)
                if (merge and type(wo) is FusedLinear and wo.lora_r == 0 and wo.weight.shape[0] % 16 == 0
                        and K % 512 == 0 and B * K <= 32768 and wo.weight.shape[1] == K):
                    # partials only: the split merge runs in the o-projection's prologue
                    return ops.native().decode_attn_partials(q, self.kv.k[i], self.kv.v[i], pos, sl, max_len,
                                                             1.0 / math.sqrt(c.head_dim), 1, bt)
                return ops.native().decode_attn(q, self.kv.k[i], self.kv.v[i], pos, sl, max_len,
                                                1.0 / math.sqrt(c.head_dim), 1, bt, cnt)
            return dops.decode_attention(qkv, m.rope_cos, m.rope_sin, self.kv.k[i], self.kv.v[i], pos, sl,
                                         c.n_heads, c.n_kv_heads, c.head_dim, max_len, bt, cnt)

        def qkv_fn(i, delta, h, gamma, layer):
            # QKV GEMM with the RoPE/cache-append epilogue; 1-2 rows also with the RMSNorm prologue
            # (one launch), more rows after the RMSNorm kernel
            if not (_ROPE_FUSED and self.tp is None and c.head_dim == 128
                    and type(layer.wqkv) is FusedLinear and layer.wqkv.lora_r == 0):
                return None
            rope = (layer.wqkv.weight, m.rope_cos, m.rope_sin, pos, sl, self.kv.k[i], self.kv.v[i],
                    c.n_heads, c.n_kv_heads, bt)
            if _NORM_FUSED:
                r = ops.qkv_rope_linear(delta, h, gamma, c.norm_eps, *rope)
                if r is not None:
                    return r
            if not ops.qkv_rope_ok(h, rope[0], rope[1], rope[2], rope[5], rope[6], rope[7], rope[8], False):
                return None
            if delta is None:
                xn = ops.rms_norm(h, gamma, c.norm_eps)
            else:
                xn, h = ops.add_rms_norm(delta, h, gamma, c.norm_eps)
            q, _ = ops.qkv_rope_linear(None, xn, None, c.norm_eps, *rope)
            return q, h

        xn = self._layers(x, attn, qkv_fn)
        return self._logits(xn)

    def _buckets(self, B: int, max_len: int) -> tuple[int, int]:
        bb = 1
        while bb < B:
            bb *= 2
        bb = min(bb, self.max_batch)
        ns, cap = (max_len + 255) // 256, (self.max_seq + 255) // 256
        nb = 1
        while nb < ns:
            nb *= 2
        return bb, min(nb, cap) * 256

    def _decode_graphed(self, slots: list[int], tokens: torch.Tensor, max_len: int) -> torch.Tensor:
        B = len(slots)
        bb, kl = self._buckets(B, max_len)
        entry = self._graphs.get((bb, kl))
        if entry is None:
            entry = self._capture(bb, kl)
        inp, out, graph, host = entry
        # the previous step's copy from ``host`` has completed: its logits were
        # read back (sampling) before this step was scheduled
        host[0, :B] = tokens.to("cpu", torch.long)
        host[1, :B] = torch.tensor([self.lens[s] for s in slots])
        host[2, :B] = torch.tensor(slots)
        host[0, B:] = 0
        host[1, B:] = 0
        host[2, B:] = self.scratch_slot
        inp.copy_(host, non_blocking=True)
        graph.replay()
        return out

    def _capture(self, bb: int, kl: int):
        inp = torch.zeros(3, bb, dtype=torch.long, device=self.device)
        inp[2].fill_(self.scratch_slot)  # warm-up / capture traffic goes to the scratch slot
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):  # library handles / workspace set up outside capture
                self._decode_body(inp, kl)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(graph, pool=self._pool, capture_error_mode="thread_local"):
            out = self._decode_body(inp, kl)
        host = torch.empty(3, bb, dtype=torch.long, pin_memory=True)
        self._graphs[(bb, kl)] = (inp, out, graph, host)
        log.debug("captured decode graph: batch %d, key bound %d", bb, kl)
        return self._graphs[(bb, kl)]

    # ------------------------------------------------------------------ scheduling
    # ------------------------------------------------------------------ embeddings
    @torch.no_grad()
    def _embed_now(self, prompts: list[list[int]]) -> torch.Tensor:
        if self.tp is not None:
            raise NotImplementedError("embeddings are served by single-GPU engines")
        out = []
        for ids in prompts:
            if not ids:
                raise ValueError("empty input")
            if len(ids) >= self.max_seq:
                raise ValueError(f"input of {len(ids)} tokens exceeds max_seq {self.max_seq}")
            t = torch.tensor([ids], dtype=torch.long, device=self.device)
            h = self.model.hidden_states(t).float()  # [S, H], final RMSNorm applied (no KV cache touched)
            out.append(torch.nn.functional.normalize(h.mean(0), dim=0))
        return torch.stack(out).cpu()

    def embed(self, prompts: list[list[int]]) -> torch.Tensor:
        """Sentence embeddings [n, hidden] (f32, unit norm): the mean of the final
        normed hidden states over each input's tokens.  With the background loop
        running the pass runs on the engine thread between decode steps (it shares
        the model's kernels and workspaces with generation); otherwise inline."""
        if self._thread is None:
            return self._embed_now(prompts)
        box, ev = {}, threading.Event()

        def task():
            try:
                box["out"] = self._embed_now(prompts)
            except Exception as e:  # noqa: BLE001
                box["err"] = e
            ev.set()

        with self._cv:
            self._tasks.append(task)
            self._cv.notify()
        ev.wait()
        if "err" in box:
            raise box["err"]
        return box["out"]

    def _run_tasks(self) -> None:
        with self._lock:
            tasks, self._tasks = self._tasks, []
        for t in tasks:
            t()

    def submit(self, prompt: list[int], params: SamplingParams | None = None) -> Request:
        r = Request(next(self._ids), list(prompt), params or SamplingParams())
        with self._cv:
            self.waiting.append(r)
            self._cv.notify()
        return r

    def stats(self) -> dict:
        """Cumulative serving metrics: TTFT / request latency means, prefill and
        decode throughput (tokens/s of engine wall time)."""
        n = max(self.finished, 1)
        return {"requests_finished": self.finished, "tokens_generated": self.tokens_generated,
                "mean_ttft_s": self.ttft_sum / n, "mean_latency_s": self.latency_sum / n,
                "prefill_tokens_per_s": self.prefill_tokens / self.prefill_s if self.prefill_s else 0.0,
                "decode_tokens_per_s": self.decode_tokens / self.decode_s if self.decode_s else 0.0,
                "decode_steps": self.steps}

    def _finish(self, r: Request, reason: str):
        r.finish_reason = reason
        r.t_done = time.perf_counter()
        self.finished += 1
        self.latency_sum += r.t_done - r.t_submit
        if r.t_first is not None:
            self.ttft_sum += r.t_first - r.t_submit
        if r.slot >= 0:
            self.kv.release(r.slot)
            self.free_slots.append(r.slot)
            self.active.pop(r.slot, None)
            r.slot = -1
        r.done.set()

    def _accept(self, r: Request, tok: int):
        if r.t_first is None:
            r.t_first = time.perf_counter()
        r.output.append(tok)
        self.tokens_generated += 1
        p = r.params
        if tok in self.eos_ids or tok in p.stop_ids:
            self._finish(r, "stop")
        elif len(r.output) >= p.max_new_tokens:
            self._finish(r, "length")
        elif self.lens[r.slot] + 1 >= self.kv.capacity(r.slot):
            self._finish(r, "length")

    def enable_tp_sync(self) -> None:
        """Server mode of a tensor-parallel group: requests arrive on group rank 0
        only; every ``step`` rank 0 broadcasts the requests it admits (prompt +
        sampling params, usually an empty list) and the other ranks, running
        ``follow()``, admit the same requests into the same slots.  The schedule
        is deterministic from there on (identical logits on every rank)."""
        if self.tp is None:
            return
        self.tp_sync = True
        self._tp_stop = False

    def _sync_admit(self, admit: list, stopping: bool = False) -> list:
        """``stopping`` (rank 0): broadcast the stop sentinel instead of admissions.  It is
        an argument, not a read of ``self._stop``: a stop() arriving mid-step must not turn
        this step's broadcast into the sentinel while rank 0 still runs the step's
        collectives (the followers would have left them)."""
        import torch.distributed as dist

        src = dist.get_global_rank(self.tp.group, 0)
        dev = self.device if dist.get_backend(self.tp.group) == "nccl" else torch.device("cpu")
        if self.tp.rank == 0:
            payload = [None if stopping else [(r.prompt, r.params) for r in admit]]
            dist.broadcast_object_list(payload, src=src, group=self.tp.group, device=dev)
            return admit
        payload = [None]
        dist.broadcast_object_list(payload, src=src, group=self.tp.group, device=dev)
        if payload[0] is None:
            self._tp_stop = True
            return []
        mirrored = []
        for prompt, params in payload[0]:
            r = Request(next(self._ids), list(prompt), params)
            r.slot = self.free_slots.pop(0)
            self.kv.reserve(r.slot, len(r.prompt) + params.max_new_tokens)
            mirrored.append(r)
        return mirrored

    def follow(self) -> None:
        """Non-zero ranks of a TP serving group: mirror rank 0's schedule until it
        stops (``enable_tp_sync`` first)."""
        self.enable_tp_sync()
        while not self._tp_stop:
            self.step()

    def step(self) -> bool:
        """Admit + prefill waiting requests into free slots, then one decode step
        for the running batch.  Returns False when there is nothing to do."""
        with self._lock:
            admit, rejected = [], []
            while self.waiting and self.free_slots:
                r = self.waiting[0]
                need = len(r.prompt) + r.params.max_new_tokens
                if not self.kv.fits_at_all(need):  # larger than the whole KV pool
                    self.waiting.pop(0)
                    rejected.append(r)
                    continue
                if not self.kv.can_reserve(need):  # paged pool full: wait for finishing requests
                    break
                self.waiting.pop(0)
                r.slot = self.free_slots.pop(0)
                self.kv.reserve(r.slot, need)
                admit.append(r)
        for r in rejected:
            r.error = f"request needs {len(r.prompt) + r.params.max_new_tokens} KV positions, more than the pool"
            self._finish(r, "error")
        if getattr(self, "tp_sync", False):
            admit = self._sync_admit(admit)
        # admitted prompts are prefilled together, in groups of at most
        # prefill_tokens tokens (bounds the activation memory of one pass)
        groups, cur, ntok = [], [], 0
        for r in admit:
            if cur and ntok + len(r.prompt) > self.prefill_budget:
                groups.append(cur)
                cur, ntok = [], 0
            cur.append(r)
            ntok += len(r.prompt)
        if cur:
            groups.append(cur)
        for grp in groups:
            try:
                t0 = time.perf_counter()
                logits = self.prefill_batch([r.slot for r in grp], [r.prompt for r in grp])
                for r in grp:
                    self.active[r.slot] = r
                toks = self._sample(logits, grp, first=True)
                self.prefill_s += time.perf_counter() - t0
                for r, tok in zip(grp, toks):
                    self.prefill_tokens += len(r.prompt)
                    self._accept(r, tok)
            except Exception as e:  # noqa: BLE001
                log.exception("prefill failed")
                for r in grp:
                    self.active.pop(r.slot, None)
                    r.error = str(e)
                    self._finish(r, "error")
        if not self.active:
            return bool(admit)
        slots = sorted(self.active)
        reqs = [self.active[s] for s in slots]
        t0 = time.perf_counter()
        tokens = torch.tensor([r.output[-1] for r in reqs], dtype=torch.long)
        logits = self.decode(slots, tokens)
        self.steps += 1
        nxt = self._sample(logits, reqs)
        self.decode_s += time.perf_counter() - t0  # includes the sampling read-back (a sync)
        self.decode_tokens += len(reqs)
        for r, t in zip(reqs, nxt):
            self._accept(r, int(t))
        return True

    @staticmethod
    def _sample(logits: torch.Tensor, reqs, first: bool = False) -> list[int]:
        """One batched draw for every row of ``logits`` with each request's own
        temperature / top-k / top-p; per-request RNG stream keyed by (seed, token
        index), so draws do not depend on batching.  One host read-back."""
        ps = [r.params for r in reqs]
        steps = [0 if first else len(r.output) for r in reqs]
        return dops.sample_rows(logits[:len(reqs)], [p.temperature for p in ps], [p.top_p for p in ps],
                                [p.top_k for p in ps], [p.seed for p in ps], steps).tolist()

    def generate(self, prompts: list[list[int]], max_new_tokens: int = 32, temperature: float = 0.0,
                 top_p: float = 1.0, top_k: int = 0, stop_ids=(), seed: int = 0) -> list[list[int]]:
        """Synchronous batched generation (continuous batching when
        len(prompts) > max_batch)."""
        if self._thread is not None:
            reqs = [self.submit(p, SamplingParams(max_new_tokens, temperature, top_p, top_k, tuple(stop_ids), seed))
                    for p in prompts]
            for r in reqs:
                r.done.wait()
            return [r.output for r in reqs]
        reqs = [self.submit(p, SamplingParams(max_new_tokens, temperature, top_p, top_k, tuple(stop_ids), seed))
                for p in prompts]
        while not all(r.done.is_set() for r in reqs):
            self.step()
        return [r.output for r in reqs]

    # ------------------------------------------------------------------ background loop (server)
    def start(self):
        if self._thread is not None:
            return
        self._stop = False

        def loop():
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
            sync = getattr(self, "tp_sync", False)
            while True:  # leaves only through the stop branch, which always tells the followers
                with self._cv:
                    while not self._stop and not self.waiting and not self.active and not self._tasks:
                        self._cv.wait(timeout=0.5)
                        if sync:  # idle heartbeat: followers wait inside a broadcast
                            break
                if self._tasks:
                    self._run_tasks()
                if self._stop:
                    if sync:
                        self._sync_admit([], stopping=True)  # tells the followers to stop
                    break
                try:
                    self.step()
                except Exception:  # noqa: BLE001
                    log.exception("engine step failed")
                    for r in list(self.active.values()):
                        r.error = "engine failure"
                        self._finish(r, "error")

        self._thread = threading.Thread(target=loop, name="mxllm-engine", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop = True
        with self._cv:
            self._cv.notify_all()
        if self._thread is not None:
            self._thread.join(timeout=10)
        self._thread = None


@torch.no_grad()
def merge_lora_(model) -> None:
    """Fold LoRA adapters into the base weights (W += s * B @ A) for serving."""
    for mod in model.modules():
        if getattr(mod, "lora_r", 0) > 0:
            delta = mod.scaling * (mod.lora_b.float() @ mod.lora_a.float())
            mod.weight += delta.to(mod.weight.dtype)
            mod.lora_r = 0
            del mod.lora_a
            del mod.lora_b
            if hasattr(mod, "wbt"):
                del mod.wbt
            if hasattr(mod, "wxt"):
                del mod.wxt
