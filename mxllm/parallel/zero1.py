"""Sharded-optimizer data parallel (ZeRO-1 style) on the bucketed DDP machinery.

Plain DDP keeps the full fp32 master + Adam moments on every rank, so the
fused AdamW streams 16-28 B/param on every GPU no matter how many there are
(8B full fine-tune: ~43 ms of a ~215 ms step).  Here the same
gradient-production-ordered buckets (mxllm/parallel/ddp.py) are
REDUCE-SCATTERED instead of all-reduced, the rank runs AdamW over its 1/N
slice of every bucket only, and the updated bf16 slices are ALL-GATHERED back
into the flat parameter buffer — the same link bytes as one all-reduce
(reduce-scatter + all-gather), 1/N of the optimizer traffic and 1/N of the
fp32 state (8B at N=8: 12 GB instead of 96 GB per GPU).

  * ownership: rank r owns elements [s + r L/N, s + (r+1) L/N) of every
    bucket [s, s+L) (buckets are multiples of 64 N elements), laid out
    back to back in compact per-rank buffers (grad shard bf16, master/m/v fp32,
    bf16 param shard) so the optimizer is still ONE fused AdamW launch;
  * backward: each bucket's reduce-scatter launches asynchronously from the
    post-accumulate-grad hooks straight into the compact grad shard — RCCL on
    its own stream, overlapped with the rest of backward;
  * after the optimizer the all-gathers are launched asynchronously in FORWARD
    order (the flat buffer is in backward order, so the last bucket first), and
    the model waits per layer (``Llama.param_wait`` hook) — the next forward
    starts as soon as its first layer's parameters have arrived;
  * the full flat grad buffer is cleared bucket by bucket once its
    reduce-scatter has completed (the dW GEMMs accumulate into it, beta = 1) --
    unless the trainer's gradients are "fresh" (every gradient op overwrites its
    slot on the step's first micro-batch: nothing to clear).
Reference: the reference claims DDP fine-tuning (README.md:7) and has none.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist

from .ddp import DDP
from .flat import FlatParams

log = logging.getLogger("mxllm.zero1")


class Zero1(DDP):
    def __init__(self, flat: FlatParams, *, bucket_mb: float = 128.0, first_bucket_mb: float = 16.0,
                 process_group=None):
        super().__init__(flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb, process_group=process_group,
                         enabled=True)
        w = self.world
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        off = 0
        self.cslices = []  # per bucket: (compact start, shard length)
        for b in self.buckets:
            L = b.end - b.start
            if L % w:
                raise ValueError(f"bucket of {L} elements is not divisible by world {w} (FlatParams align)")
            self.cslices.append((off, L // w))
            off += L // w
        self.shard_numel = off
        dev = flat.device
        self.gshard = torch.zeros(off, dtype=flat.grads.dtype, device=dev)
        self.pshard = torch.empty(off, dtype=flat.params.dtype, device=dev)
        with torch.no_grad():
            for b, (cs, n) in zip(self.buckets, self.cslices):
                own = b.start + self.rank * n
                self.pshard[cs:cs + n].copy_(flat.params[own:own + n])
        self.master = self.pshard.float() if flat.params.dtype != torch.float32 else self.pshard
        self._ag_work: list = [None] * len(self.buckets)
        # clear each bucket of the full gradient buffer once its reduce-scatter is done (the dW GEMMs
        # accumulate into it); False when every gradient op overwrites its slot on the step's first
        # micro-batch (the trainer's "fresh" gradients)
        self.clear_grads = True
        self._launched: set[int] = set()  # bucket indices reduce-scattered this step
        self._param_slot_bucket = {id(p): bi for p, bi in zip(flat.param_list, self._param_bucket)}
        log.info("ZeRO-1: %d buckets, optimizer shard %.1f M of %.1f M elements (world %d)", len(self.buckets),
                 off / 1e6, flat.numel / 1e6, w)

    @property
    def bytes_per_step(self) -> int:
        return self.flat.numel * self.flat.grads.element_size()

    def _launch(self, b):
        self._launched.add(b.index)
        cs, n = self.cslices[b.index]
        g = self.flat.grads[b.start:b.end]
        out = self.gshard[cs:cs + n]
        if self.world > 1:
            b.work = self.comm.reduce_scatter(out, g, async_op=True)
        else:
            out.copy_(g)
            b.work = None
            if self.clear_grads:
                g.zero_()

    def finish(self) -> float:
        """Wait for every bucket's reduce-scatter, clear the full grad buffer
        behind it, return the gradient scale (1/world)."""
        for b in self.buckets:
            if b.index not in self._launched and self._sync:
                self._launch(b)  # hooks did not all fire (unused parameters)
        timing = self._timing and torch.cuda.is_available() and self.flat.grads.is_cuda
        if timing:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if self.clear_grads:
                    self.flat.grads[b.start:b.end].zero_()  # dW GEMMs accumulate (beta 1) next step
            b.work = None
            b.pending = b.expected
            b.seen.clear()
        self._launched.clear()
        if timing:
            e1.record()
            self._last_events = (e0, e1)
        from .comm import verify

        verify(self.comm)  # peer path: a timed-out exchange stops the step before AdamW reads the shard
        return 1.0 / self.world

    # ------------------------------------------------------------ parameters
    def gather_params(self):
        """Launch the all-gathers of the updated bf16 shards, forward order first."""
        for b in reversed(self.buckets):
            cs, n = self.cslices[b.index]
            dst = self.flat.params[b.start:b.end]
            if self.world > 1:
                self._ag_work[b.index] = self.comm.all_gather(dst, self.pshard[cs:cs + n], async_op=True)
            else:
                dst.copy_(self.pshard[cs:cs + n])

    def wait_params(self, params=None):
        """Make the compute stream wait for the all-gathers holding ``params``
        (all of them when None).  No host synchronisation."""
        if params is None:
            idx = range(len(self.buckets))
        else:
            idx = sorted({self._param_slot_bucket[id(p)] for p in params if id(p) in self._param_slot_bucket})
        for i in idx:
            w = self._ag_work[i]
            if w is not None:
                w.wait()
                self._ag_work[i] = None

    def broadcast_params(self, src: int = 0):
        if self.world > 1:
            self.comm.broadcast(self.flat.params, src=src)
        with torch.no_grad():
            for b, (cs, n) in zip(self.buckets, self.cslices):
                own = b.start + self.rank * n
                self.pshard[cs:cs + n].copy_(self.flat.params[own:own + n])
            if self.master is not self.pshard:
                self.master.copy_(self.pshard)

    def full_master(self) -> torch.Tensor:
        """The full fp32 master in flat layout, assembled from every rank's
        shards (collective: all ranks call it; tests / export)."""
        full = torch.zeros(self.flat.numel, dtype=torch.float32, device=self.flat.device)
        for b, (cs, n) in zip(self.buckets, self.cslices):
            src = self.master[cs:cs + n].float().contiguous()
            if self.world > 1:
                self.comm.all_gather(full[b.start:b.end], src)
            else:
                full[b.start:b.end].copy_(src)
        return full
