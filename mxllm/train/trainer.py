"""Training step: forward -> fused CE -> backward (bucketed RCCL all-reduce
overlapped via DDP hooks) -> grad-norm clip -> fused AdamW over flat buffers.

This is the real version of the reference's simulated ``process_batch``
(reference src/utils.py:12-23): the loss is computed from the
model's own logits and gradients flow into an optimizer step.
"""
from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass

import torch

from .. import ops
from ..parallel.ddp import DDP
from ..parallel.flat import FlatParams, production_order
from ..parallel.runtime import DistEnv
from ..utils.profiling import range_

log = logging.getLogger("mxllm.train")


@dataclass
class OptimConfig:
    lr: float = 1e-4
    beta1: float = 0.9
    beta2: float = 0.95
    eps: float = 1e-8
    weight_decay: float = 0.0
    grad_clip: float = 1.0
    warmup_steps: int = 0
    total_steps: int = 0  # 0 = constant lr after warmup

    def lr_at(self, step: int) -> float:
        if self.warmup_steps and step <= self.warmup_steps:
            return self.lr * step / self.warmup_steps
        if self.total_steps and step > self.warmup_steps:
            prog = min(1.0, (step - self.warmup_steps) / max(1, self.total_steps - self.warmup_steps))
            return self.lr * 0.5 * (1.0 + math.cos(math.pi * prog))
        return self.lr


def _overlap_default() -> bool:
    return os.environ.get("MXLLM_OVERLAP_ADAMW", "1") != "0"


def _fresh_guard(p):
    """Tensor hook (runs before AccumulateGrad adds ``g`` into ``p.grad``): a slot still
    flagged fresh holds last step's gradient -> zero it first (fp32 mode: the flat fold in
    ``sync_grads_from_params`` already copies instead of adding)."""
    def hook(g):
        if getattr(p, "_mx_grad_fresh", False) and getattr(p, "_mx_grad32", None) is None and p.grad is not None:
            p.grad.zero_()
            p._mx_grad_fresh = False
        return g
    return hook


class Trainer:
    def __init__(self, model: torch.nn.Module, env: DistEnv, optim: OptimConfig | None = None, *,
                 bucket_mb: float = 128.0, first_bucket_mb: float = 16.0, broadcast_init: bool = False,
                 shard_optimizer: bool = False, overlap_optimizer: bool | None = None,
                 grad_dtype: torch.dtype | str | None = None):
        """``shard_optimizer``: ZeRO-1 (mxllm/parallel/zero1.py) — gradients are
        reduce-scattered, each rank updates its 1/N slice, parameters are
        all-gathered back.  At world 1 it is plain DDP (nothing to shard).

        ``overlap_optimizer`` (None = auto: GPU, full fine-tuning, DDP): the fused
        AdamW is issued per forward parameter group on a side stream at the end of
        the step and the NEXT forward waits per layer (see ``_launch_overlapped``).

        ``grad_dtype``: dtype of the flat gradient buffer = the dtype gradients are
        ACCUMULATED (micro-batches) and ALL-REDUCED in.  ``torch.float32``: fp32
        accumulation and fp32 ring reduction (the dW GEMMs write fp32 output);
        default: the parameter dtype (bf16)."""
        self.model = model
        self.env = env
        self.opt = optim or OptimConfig()
        named = production_order(model, [(n, p) for n, p in model.named_parameters() if p.requires_grad])
        world = env.world_size
        self.zero1 = None
        if isinstance(grad_dtype, str):
            grad_dtype = {"fp32": torch.float32, "float32": torch.float32, "bf16": None, "bfloat16": None}[grad_dtype]
        if shard_optimizer and world > 1:
            from ..parallel.zero1 import Zero1

            self.flat = FlatParams(named, align=64 * world, grad_dtype=grad_dtype, reverse=False)
            self.ddp = self.zero1 = Zero1(self.flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb)
            self._master = self.zero1.master
            if getattr(model, "param_wait", "absent") is None:
                model.param_wait = self.zero1.wait_params  # per-layer wait in the next forward
        else:
            self.flat = FlatParams(named, grad_dtype=grad_dtype, reverse=False,
                                   split_master=os.environ.get("MXLLM_SPLIT_MASTER", "1") != "0")
            self.ddp = DDP(self.flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb)
            self._master = self.flat.master
        if broadcast_init:
            self.ddp.broadcast_params(0)
        self._sync_adapters()
        self.m = torch.zeros(self._master.numel(), dtype=torch.float32, device=self._master.device)
        self.v = torch.zeros_like(self.m)
        self.step_num = 0
        self.last_grad_norm: torch.Tensor | None = None
        # ---- optimizer / next-forward overlap
        self._chunks: list[tuple[int, int]] | None = None
        self._pending: list = []
        self._hold = None
        lora = bool(getattr(model, "lora", False))
        if overlap_optimizer is None:
            overlap_optimizer = (_overlap_default() and self.flat.device.type == "cuda" and self.zero1 is None
                                 and (not lora or os.environ.get("MXLLM_LORA_OVERLAP_ADAMW", "0") == "1"))
        # LoRA: opt-in -- the headline measured 1.5 ms/step SLOWER overlapped (860.5 / 861.5 vs 858.7 /
        # 860.4 ms same box, profiles/r6m/): the update is 2.6 ms of HBM streaming that time-shares the
        # CUs of the forward's GEMMs instead of hiding under them
        self._chunk_copies: list | None = None  # LoRA: per chunk, the adapter -> wbuf copy launch
        if overlap_optimizer and self.zero1 is None and getattr(model, "param_wait", "absent") is None:
            self._chunks = self._forward_chunks()
            if self._chunks is not None and lora:
                self._chunk_copies = self._adapter_chunk_copies()
                if self._chunk_copies is None:
                    self._chunks = None
            if self._chunks is not None:
                self._side = torch.cuda.Stream(self.flat.device) if self.flat.device.type == "cuda" else None
                cus = os.environ.get("MXLLM_ADAMW_CUS", "")
                if self._side is not None and cus:
                    # the overlapped AdamW confined to a CU subset (the forward keeps the rest)
                    self._side = cu_masked_stream(self.flat.device, cus)
                model.param_wait = self._param_wait
                if self._side is not None and os.environ.get("MXLLM_STEP_PRIORITY", "0") == "1":
                    # forward/backward on a HIGH-priority stream, the overlapped AdamW on the
                    # lowest: as AdamW workgroups retire, the dispatcher hands the freed CUs to
                    # the step's kernels first (AdamW fills the gaps instead of delaying them)
                    least, greatest = torch.cuda.Stream.priority_range()
                    self._side = torch.cuda.Stream(self.flat.device, priority=least)
                    self._main = torch.cuda.Stream(self.flat.device, priority=greatest)
        self.overlap_optimizer = self._chunks is not None
        # MXLLM_ADAMW_LAG=L > 0: only chunks [0, L) are issued at the end of the step; the next
        # forward issues chunk k + L when it reaches group k, ordered after its own progress, so
        # the update is spread over the forward instead of saturating HBM under its first layers
        self._lag = int(os.environ.get("MXLLM_ADAMW_LAG", "0") or 0)
        self._deferred: list = []
        if not hasattr(self, "_main"):
            self._main = None
        # "fresh" gradients: every gradient of the step is formed by an op that can
        # OVERWRITE its flat slot (dW GEMMs with beta 0, the RMSNorm / embedding
        # kernels' accum_grad), so AdamW need not zero the gradient buffer behind
        # itself (2-4 B/param less HBM traffic per step); under ZeRO-1 the full
        # gradient buffer is then not cleared behind each reduce-scatter either (8B:
        # a 16 GB memset per step).  GPU kernels only; not with LoRA (its kernels
        # accumulate) or parameters used twice (tied embeddings: autograd sums)
        self.fresh_grads = (os.environ.get("MXLLM_FRESH_GRADS", "1") != "0" and self.flat.device.type == "cuda"
                            and not getattr(model, "lora", False)
                            and not any(getattr(p, "_mx_no_direct", False) for p in self.flat.param_list))
        if self.zero1 is not None:
            self.zero1.clear_grads = not self.fresh_grads
        # ---- fused clip norm: the dW GEMMs that write a gradient first (beta 0) also write one sum of
        # squares of the stored bf16 values per 256 x 256 tile (gemm8_sq), so the norm no longer
        # re-reads the whole gradient after the backward (8B full: 16 GB, ~2.9 ms on the critical
        # path); the rest (embedding, norm weights) is summed directly.  World 1, one micro-batch
        # (later micro-batches accumulate; at world > 1 the norm is of the reduced gradient).
        self._sq_params: list = []
        self._sq_plan: dict = {}
        self._sq_armed = False
        if (self.fresh_grads and self.opt.grad_clip and self.opt.grad_clip > 0 and self.zero1 is None
                and world == 1 and os.environ.get("MXLLM_FUSED_GRAD_NORM", "1") != "0"
                and os.environ.get("MXLLM_NORM_OVERLAP", "0") != "1"):
            regions, off = [], 0
            for p in self.flat.param_list:
                if (p.requires_grad and p.dim() == 2 and p.dtype == torch.bfloat16 and p.shape[0] % 256 == 0
                        and p.shape[1] % 256 == 0):
                    n = (p.shape[0] // 256) * (p.shape[1] // 256)
                    regions.append((p, off, n))
                    off += n
            if regions:
                self._sqbuf = torch.zeros(off, dtype=torch.float32, device=self.flat.device)
                for p, o, n in regions:
                    p._mx_sq = self._sqbuf[o:o + n]
                self._sq_params = [p for p, _, _ in regions]
        if self.fresh_grads:
            # enforce the invariant: a gradient that reaches a parameter through
            # autograd's AccumulateGrad (not an op honouring _mx_grad_fresh) would be ADDED onto
            # last step's stale slot -- zero the slot first, once, right before that accumulation
            for p in self.flat.param_list:
                if p.requires_grad:
                    p.register_hook(_fresh_guard(p))
        # ---- gradient-norm overlap: each DDP bucket's sum of squares is taken on a side
        # stream as soon as the bucket is final (after its all-reduce), under the rest of
        # the backward, instead of one pass over the whole gradient after it (8B full:
        # 16 GB, ~3 ms on the critical path); a fixed-order sum of the per-bucket values
        # gives the clip coefficient (deterministic, identical on every rank)
        self._norm_side = None
        if (self.opt.grad_clip and self.opt.grad_clip > 0 and self.zero1 is None
                and self.flat.device.type == "cuda" and os.environ.get("MXLLM_NORM_OVERLAP", "0") == "1"):
            self._norm_side = torch.cuda.Stream(self.flat.device)
            self._bsq = torch.zeros(len(self.ddp.buckets), dtype=torch.float32, device=self.flat.device)
            self.ddp.set_on_ready(self._bucket_sq_norm)

    @property
    def lowp(self):
        """The bf16 copy AdamW refreshes (None: fp32 params, or a split master whose
        high half IS the parameter buffer)."""
        if self.flat.master is self.flat.params or isinstance(self.flat.master, ops.SplitMaster):
            return None
        return self.flat.params

    def master_fp32(self) -> torch.Tensor:
        """The fp32 master weights as one tensor (flat layout; a copy when split)."""
        self.params_ready()
        return self._master.float()

    @property
    def grad_dtype(self) -> torch.dtype:
        return self.flat.grad_dtype

    # ------------------------------------------------------------------ overlap
    def _forward_chunks(self) -> list[tuple[int, int]] | None:
        """Flat-buffer ranges of the model's forward parameter groups
        (``Llama._wait_groups``: embedding, each layer + the next norm, head), in
        forward order.  The flat buffer is laid out group by group
        (``flat.production_order``), so every group is ONE contiguous range; None if
        that does not hold (the optimizer then runs as one launch)."""
        groups_fn = getattr(self.model, "_wait_groups", None)
        if groups_fn is None:
            return None
        slots = self.flat.slots
        order = sorted(range(len(slots)), key=lambda k: slots[k].offset)
        extent = {}
        for j, k in enumerate(order):  # a slot owns its alignment pad up to the next slot
            end = slots[order[j + 1]].offset if j + 1 < len(order) else self.flat.numel
            extent[k] = (slots[k].offset, end)
        slot_of = {id(p): k for k, p in enumerate(self.flat.param_list)}
        chunks, self._group_chunk = [], {}
        covered = 0
        taken: set[int] = set()  # a parameter shared by two groups belongs to the first one that uses it
        for g in groups_fn():
            ks = sorted({slot_of[id(p)] for p in g if id(p) in slot_of} - taken, key=lambda k: extent[k][0])
            if not ks:
                continue
            taken.update(ks)
            lo, hi = extent[ks[0]][0], extent[ks[-1]][1]
            if sum(extent[k][1] - extent[k][0] for k in ks) != hi - lo:
                return None  # another group's slot inside the range
            self._group_chunk[id(g)] = len(chunks)
            chunks.append((lo, hi))
            covered += hi - lo
        if covered != self.flat.numel or len(chunks) < 2:
            return None
        return chunks

    def _adapter_chunk_copies(self) -> list | None:
        """LoRA with the overlapped update: per forward chunk, ONE batched copy (csrc/kernels/misc.hip
        ``copy2d_batched``) of the chunk's adapters into their augmented GEMM buffers, issued on the
        side stream right after the chunk's AdamW, so the next forward's wait before layer i also
        covers its GEMM buffers (the one end-of-step copy of every adapter would have to wait for the
        whole update).  None when an augmented projection's adapters are not inside one chunk."""
        from ..models.llama import FusedLinear
        from ..ops.linear import copy2d_plan

        if not ops.native_available() or self.flat.device.type != "cuda":
            return None
        chunk_of = {}
        for g in self.model._wait_groups():
            k = self._group_chunk.get(id(g))
            if k is not None:
                for p in g:
                    chunk_of.setdefault(id(p), k)
        per: list[list] = [[] for _ in self._chunks]
        for mod in self.model.modules():
            if isinstance(mod, FusedLinear) and mod.augmented():
                ka, kb = chunk_of.get(id(mod.lora_a)), chunk_of.get(id(mod.lora_b))
                if ka is None or ka != kb:
                    return None
                per[ka].extend(mod.adapter_copies())
        out = []
        for pairs in per:
            if not pairs:
                out.append(None)
                continue
            rows, total = copy2d_plan(pairs)
            out.append((torch.tensor(rows, dtype=torch.int64, device=self.flat.device), total))
        return out

    def _param_wait(self, group):
        """``Llama.param_wait``: the compute stream waits for the update of the
        chunk holding ``group`` (no host synchronisation)."""
        k = self._group_chunk.get(id(group))
        if k is None or k >= len(self._pending):
            return
        if self._deferred:
            self._issue_deferred(k + self._lag, after_current=True)
        ev = self._pending[k]
        if ev is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(ev)
            self._pending[k] = None

    def params_ready(self):
        """Order the current stream after every in-flight parameter update
        (overlapped AdamW chunks, ZeRO-1 all-gathers): call before reading
        parameters outside a forward (checksums, checkpoints, export)."""
        if self.zero1 is not None:
            self.zero1.wait_params()
        if self._deferred:
            self._issue_deferred(len(self._pending), after_current=False)
        for k, ev in enumerate(self._pending):
            if ev is not None:
                torch.cuda.current_stream(self.flat.device).wait_event(ev)
                self._pending[k] = None

    def _launch_overlapped(self, gscale, **kw):
        """The fused AdamW over each forward chunk on the side stream, in forward
        order, with one event per chunk.  The NEXT forward waits for chunk i just
        before layer i, so the update of the layers it has not reached yet runs
        under its GEMMs (the update is still fully issued inside this step).
        Elementwise kernel over the same slices with the same inputs: bitwise
        identical to the one-launch update."""
        lowp = self.lowp
        side = self._side
        if side is None:  # CPU: same chunked update, in order (tests)
            for lo, hi in self._chunks:
                ops.adamw_step_(self.flat.master[lo:hi], self.flat.grads[lo:hi], self.m[lo:hi], self.v[lo:hi],
                                None if lowp is None else lowp[lo:hi], grad_scale=gscale,
                                zero_grad=not self.fresh_grads, **kw)
            return
        side.wait_stream(torch.cuda.current_stream(self.flat.device))
        self._hold = gscale  # read on the side stream: keep it alive until the next step
        if len(self._pending) != len(self._chunks):
            self._pending = [None] * len(self._chunks)
        n_now = len(self._chunks) if self._lag <= 0 else min(self._lag, len(self._chunks))
        self._deferred = [(k, gscale, kw) for k in range(n_now, len(self._chunks))]
        with torch.cuda.stream(side):
            for k in range(n_now):
                self._adamw_chunk(k, gscale, kw, side)

    def _adamw_chunk(self, k, gscale, kw, side):
        lo, hi = self._chunks[k]
        lowp = self.lowp
        ops.adamw_step_(self.flat.master[lo:hi], self.flat.grads[lo:hi], self.m[lo:hi], self.v[lo:hi],
                        None if lowp is None else lowp[lo:hi], grad_scale=gscale,
                        zero_grad=not self.fresh_grads, **kw)
        if self._chunk_copies is not None and self._chunk_copies[k] is not None:
            desc, blocks = self._chunk_copies[k]  # this chunk's adapters -> their GEMM buffers
            ops.native().copy2d_batched(desc, blocks)
        ev = torch.cuda.Event()
        ev.record(side)
        self._pending[k] = ev

    def _issue_deferred(self, upto: int, after_current: bool):
        """Issue the deferred AdamW chunks with index < ``upto`` (MXLLM_ADAMW_LAG);
        ``after_current``: the side stream first waits for the compute stream's
        current position (the forward has reached that layer)."""
        todo = [d for d in self._deferred if d[0] < upto]
        if not todo:
            return
        self._deferred = [d for d in self._deferred if d[0] >= upto]
        side = self._side
        if after_current:
            side.wait_stream(torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(side):
            for k, gscale, kw in todo:
                self._adamw_chunk(k, gscale, kw, side)

    def _bucket_sq_norm(self, b) -> None:
        """DDP on_ready callback: sum of squares of bucket ``b`` on the norm stream."""
        side = self._norm_side
        side.wait_stream(torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(side):
            if b.work is not None:
                b.work.wait()  # this stream waits for the bucket's all-reduce
            self._bsq[b.index:b.index + 1].copy_(ops.sq_norm(self.flat.grads[b.start:b.end]))

    def train_step(self, micro_batches: list[tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """One optimizer step over ``micro_batches`` [(ids, labels), ...].
        Returns the mean loss as a device tensor (no host sync)."""
        if self._main is not None:  # MXLLM_STEP_PRIORITY: the step on the high-priority stream
            cur = torch.cuda.current_stream(self.flat.device)
            self._main.wait_stream(cur)
            with torch.cuda.stream(self._main):
                out = self._train_step(micro_batches)
            cur.wait_stream(self._main)
            return out
        return self._train_step(micro_batches)

    def _train_step(self, micro_batches):
        total, scale = self.compute_grads(micro_batches)
        self.step_num += 1
        with range_("optimizer"):
            self._optimizer_step(scale)
        return total / len(micro_batches)

    def compute_grads(self, micro_batches: list[tuple[torch.Tensor, torch.Tensor]]):
        """Forward + backward of every micro-batch (gradients accumulated in the
        flat buffer, reduced across ranks by the DDP buckets).  Returns (sum of
        the micro-batch losses, scale that turns the flat gradient into the mean
        gradient) — each backward runs on loss / n, so the flat buffer holds the
        SUM over ranks of each rank's micro-batch MEAN and the scale is 1 / world
        (it used to divide by n a second time: the clip norm read n x too small
        under gradient accumulation)."""
        n = len(micro_batches)
        self.model.train()
        if self.zero1 is not None and getattr(self.model, "param_wait", None) is None:
            self.zero1.wait_params()  # model without per-layer waits: all parameters first
        if self.fresh_grads:
            for p in self.flat.param_list:
                p._mx_grad_fresh = True
        self._sq_armed = bool(self._sq_params) and n == 1
        if self._sq_params:
            if self._sq_armed:
                self._sqbuf.zero_()  # regions of gradients written another way stay 0
            for p in self._sq_params:
                p._mx_sq_done = False if self._sq_armed else None
        total = None
        for i, (ids, labels) in enumerate(micro_batches):
            last = i == n - 1
            ctx = self.ddp.no_sync() if not last else _null()
            with ctx:
                with range_("forward"):
                    loss = self.model(ids, labels)
                with range_("backward"):
                    (loss / n if n > 1 else loss).backward()
            total = loss.detach() if total is None else total + loss.detach()
        if self._deferred:  # a forward that skipped parameter groups: nothing may stay un-updated
            self._issue_deferred(len(self._pending), after_current=False)
        fired = [b.fired for b in self.ddp.buckets]
        changed = self.flat.sync_grads_from_params()
        if self.fresh_grads:
            self.flat.zero_unwritten_()
        with range_("grad_allreduce_wait"):
            scale = self.ddp.finish()
        if self._norm_side is not None and changed:
            # a gradient folded into the flat buffer after its bucket's norm was taken
            for bi in sorted({self.ddp._param_bucket[k] for k in changed}):
                if fired[bi]:
                    self._bucket_sq_norm(self.ddp.buckets[bi])
        return total, scale

    def _optimizer_step(self, scale: float):
        o = self.opt
        z = self.zero1
        grads = z.gshard if z is not None else self.flat.grads
        if o.grad_clip and o.grad_clip > 0:
            # global grad norm on device; the clip coefficient is applied inside
            # the fused AdamW kernel via grad_scale (host read only for logging)
            sq = self._fused_sq() if self._sq_armed else None
            if sq is not None:
                pass
            elif self._norm_side is not None:  # per-bucket partials taken during the backward
                torch.cuda.current_stream(self.flat.device).wait_stream(self._norm_side)
                sq = self._bsq.sum(0, keepdim=True)
            else:
                sq = ops.sq_norm(grads)
            if z is not None:
                z.comm.all_reduce(sq)  # sum of the shards' squares (stream-ordered, same communicator)
            gnorm = sq.sqrt() * scale
            self.last_grad_norm = gnorm
            coef = torch.clamp(o.grad_clip / (gnorm + 1e-6), max=1.0)
            gscale = coef * scale
        else:
            gscale = scale
        if z is not None:
            lowp = None if z.master is z.pshard else z.pshard
            ops.adamw_step_(z.master, grads, self.m, self.v, lowp, lr=o.lr_at(self.step_num), beta1=o.beta1,
                            beta2=o.beta2, eps=o.eps, weight_decay=o.weight_decay, step=self.step_num,
                            grad_scale=gscale, zero_grad=True)
            z.gather_params()  # async, forward order; the next forward waits per layer
            if getattr(self.model, "sync_adapters_", None) is not None and getattr(self.model, "lora", False):
                z.wait_params()
        elif self._chunks is not None:
            self._launch_overlapped(gscale, lr=o.lr_at(self.step_num), beta1=o.beta1, beta2=o.beta2, eps=o.eps,
                                    weight_decay=o.weight_decay, step=self.step_num)
        else:
            ops.adamw_step_(self.flat.master, grads, self.m, self.v, self.lowp, lr=o.lr_at(self.step_num),
                            beta1=o.beta1, beta2=o.beta2, eps=o.eps, weight_decay=o.weight_decay,
                            step=self.step_num, grad_scale=gscale,
                            zero_grad=not self.fresh_grads)  # else grads cleared in the same pass
        if self._chunk_copies is None or self._side is None:
            self._sync_adapters()  # (overlapped LoRA on GPU: each chunk copies its adapters after its update)
        self.flat.attach_grads()

    def _fused_sq(self):
        """Sum of squares of the whole gradient from the dW GEMMs' per-tile partials plus a direct
        pass over the slots no armed GEMM wrote (None when none did: the caller takes the full pass)."""
        done = tuple(p._mx_sq_done is True for p in self._sq_params)
        if not any(done) or any(p._mx_sq_done == "dirty" for p in self._sq_params):
            return None
        plan = self._sq_plan.get(done)
        if plan is None:
            covered = {id(p) for p, d in zip(self._sq_params, done) if d}
            big, small = [], []
            for slot, p in zip(self.flat.slots, self.flat.param_list):
                if id(p) in covered or not p.requires_grad:
                    continue
                (big if slot.numel >= (1 << 20) else small).append((slot.offset, slot.offset + slot.numel))
            plan = self._sq_plan[done] = (big, small)
        big, small = plan
        g = self.flat.grads
        parts = [self._sqbuf.sum().reshape(1)] + [ops.sq_norm(g[lo:hi]) for lo, hi in big]
        if small:
            parts.append(ops.sq_norm(torch.cat([g[lo:hi] for lo, hi in small])))
        return torch.cat(parts).sum().reshape(1)  # one fixed-order sum, not a chain of adds

    def _sync_adapters(self):
        """LoRA adapters -> their copies in the augmented GEMM weight buffers."""
        fn = getattr(self.model, "sync_adapters_", None)
        if fn is not None:
            fn()

    # ------------------------------------------------------------------ state
    @property
    def sharded_state(self) -> bool:
        """True when each rank's optimizer state differs (ZeRO-1): save every rank."""
        return self.zero1 is not None

    def state_dict(self) -> dict:
        self.params_ready()
        return {"step": self.step_num, "master": self._master, "m": self.m, "v": self.v,
                "layout": self.flat.state_dict()}

    def load_state_dict(self, sd: dict):
        self.params_ready()
        self._master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.finish_load(int(sd["step"]))

    def finish_load(self, step: int):
        """After master/m/v were written in place (checkpoint.load): set the step
        and rebuild the compute-dtype parameters from the fp32 master."""
        self.step_num = int(step)
        z = self.zero1
        if z is not None:
            if z.master is not z.pshard:
                z.pshard.copy_(z.master)
            z.gather_params()
            z.wait_params()
        elif self.flat.master is not self.flat.params and not isinstance(self.flat.master, ops.SplitMaster):
            self.flat.params.copy_(self.flat.master)
        self._sync_adapters()


_MASKED: dict = {}


def cu_masked_stream(device: torch.device, spec: str) -> torch.cuda.ExternalStream:
    """A stream confined to a CU subset (csrc/bindings.cpp ``cu_masked_stream``).
    ``spec``: ``first:K`` (CU bits 0..K-1), ``mod8:K`` (K of every 8 consecutive
    bits), ``stride:K`` (every K-th bit) or a hex mask ``0x...``."""
    from ..ops._ext import native

    key = (str(device), spec)
    if key in _MASKED:  # one HIP stream (and hardware queue) per mask for the process
        return _MASKED[key]
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    if spec.startswith("0x"):
        bits = int(spec, 16)
        on = [i for i in range(ncu) if (bits >> i) & 1]
    else:
        kind, k = spec.split(":")
        k = int(k)
        pick = {"first": lambda i: i < k, "mod8": lambda i: i % 8 < k, "stride": lambda i: i % k == 0}[kind]
        on = [i for i in range(ncu) if pick(i)]
    if not on:
        raise ValueError(f"CU mask {spec!r} selects no CU")
    words = [0] * ((ncu + 31) // 32)
    for i in on:
        words[i // 32] |= 1 << (i % 32)
    words = [w - (1 << 32) if w >= 1 << 31 else w for w in words]  # int64 schema, low 32 bits used
    ptr = native().cu_masked_stream(device.index if device.index is not None else torch.cuda.current_device(),
                                    words)
    log.info("AdamW stream on %d of %d CUs (%s)", len(on), ncu, spec)
    _MASKED[key] = torch.cuda.ExternalStream(ptr, device=device)
    return _MASKED[key]


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def timed(fn, sync_device: torch.device | None = None):
    t0 = time.perf_counter()
    r = fn()
    if sync_device is not None and sync_device.type == "cuda":
        torch.cuda.synchronize(sync_device)
    return r, time.perf_counter() - t0
