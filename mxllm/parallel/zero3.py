"""ZeRO-3 / fully-sharded data parallel for full fine-tuning.

Llama-3.1-70B full fine-tuning needs 16 B/param = 1,129 GB of state: it only
fits an 8 x 288 GB MI355X node sharded (141 GB of state per GPU).  Design:

  * units: the model is cut into flat parameter units — the embedding, each
    transformer layer's four projection matrices, the LM head — plus one small
    always-resident unit holding every RMSNorm weight.  Each unit is a flat
    bf16 buffer split evenly over the ranks; a rank keeps only its slice
    (bf16 compute shard + fp32 master + Adam m, v + fp32 grad shard), all as
    views into ONE flat per-rank buffer each, so the optimizer is one fused
    AdamW launch per step.
  * forward: a unit is all-gathered (``all_gather_into_tensor`` over RCCL /
    xGMI: each rank receives 7/8 of a 1.7 GB layer) just before use, with the
    NEXT unit's gather already in flight, and released after use.
  * autograd never keeps a gathered weight alive: a ``saved_tensors_hooks``
    pair saves a (unit, offset, shape, stride) handle instead of any tensor
    that lives in a gathered buffer.  An identity autograd node at every
    unit's output (``_PreBackward``) runs first in backward: it re-gathers the
    unit (waiting on the prefetch issued one unit earlier), prefetches the unit
    below and attaches the unit's gradient buffer.
  * gradients: the projection backward writes dW straight into a per-unit
    flat bf16 gradient buffer (``param_weight_grad``, beta 0: no zero fill,
    no concatenation copy).  When the unit's last gradient lands, the buffer is
    reduce-scattered ASYNCHRONOUSLY on a second communicator (so gathers and
    reduce-scatters of neighbouring units use both directions of the xGMI
    links concurrently); at most ``max_inflight`` reduce-scatters are
    outstanding, and each finished one is folded into the fp32 grad shard on
    the compute stream (a dependency, never a host wait).
  * activation checkpointing: a layer's forward runs under no_grad keeping
    only its (x, h) inputs; its backward re-gathers the unit, recomputes the
    layer and back-propagates through it (one gather serves both).
  * the model is built on the meta device and materialised unit by unit with
    a per-unit seed, so no rank ever holds the full 141 GB model.
  * ``emulate_world=W`` (one process): the rank holds world-W shard sizes and
    a gather tiles the local shard W times, a reduce-scatter sums the W
    slices — the per-rank memory footprint and local traffic of a W-GPU run
    without its link traffic (the 80-layer config-4 sizing proxy).
Reference parity: none — the reference advertises 70B fine-tuning
(README.md:1-3) with no training code.
"""
from __future__ import annotations

import logging
import math
import os
from collections import deque

import torch
import torch.distributed as dist

from .. import ops
from .runtime import DistEnv

log = logging.getLogger("mxllm.zero3")
ALIGN = 64
_EMPTY = {}


def _empty(dtype, device):
    key = (dtype, str(device))
    if key not in _EMPTY:
        _EMPTY[key] = torch.empty(0, dtype=dtype, device=device)
    return _EMPTY[key]


def _realize_on(model, device):
    """Swap every meta parameter for an empty real parameter on ``device`` (the
    unit machinery points .data at gathered views later); real rope tables."""
    import torch.nn as nn

    from ..ops import reference as ref

    model._meta_shapes = {}
    for mname, mod in model.named_modules():
        for pname, p in list(mod._parameters.items()):
            if p is None:
                continue
            full = f"{mname}.{pname}" if mname else pname
            model._meta_shapes[full] = tuple(p.shape)
            mod._parameters[pname] = nn.Parameter(torch.empty(0, dtype=torch.bfloat16, device=device))
    cfg = model.cfg
    if cfg.tie_embeddings:
        model.tok_emb._mx_no_direct = True
    cos, sin = ref.rope_tables(min(cfg.max_seq_len, 131072), cfg.head_dim, cfg.rope_theta, cfg.rope_scaling, device)
    model.rope_cos, model.rope_sin = cos, sin


def unit_layout(model):
    """[(name, [(param_name, param, shape)], resident)] — norms | emb | layers | head."""
    named = dict(model.named_parameters())
    shp = model._meta_shapes

    def ent(n):
        return (n, named[n], shp[n])

    units = [("norms", [ent(n) for n in named if n.endswith("norm")], True), ("emb", [ent("tok_emb")], False)]
    for i in range(len(model.layers)):
        units.append((f"layer{i}", [ent(f"layers.{i}.{k}.weight") for k in ("wqkv", "wo", "wgu", "wd")], False))
    if model.lm_head is not None:
        units.append(("head", [ent("lm_head")], False))
    return units


def init_unit_full(uid, names, numels, full_numel, seed, device):
    """Deterministic full flat init of one unit (norms = 1, weights ~ N(0, 0.02))."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed * 100003 + uid)
    full = torch.zeros(full_numel, dtype=torch.bfloat16, device=device)
    off = 0
    for name, n in zip(names, numels):
        if name.endswith("norm"):
            full[off:off + n].fill_(1.0)
        else:
            full[off:off + n].normal_(0.0, 0.02, generator=gen)
        off += n
    return full


def init_full_state(cfg, seed, device) -> dict:
    """The named full weights a Zero3Trainer with ``seed`` starts from (tests/export)."""
    from ..models.llama import Llama

    model = Llama(cfg, device="meta", init=False)
    _realize_on(model, device)
    out = {}
    for k, (_, ents, _) in enumerate(unit_layout(model)):
        names = [e[0] for e in ents]
        numels = [math.prod(e[2]) for e in ents]
        full = init_unit_full(k, names, numels, sum(numels), seed, device)
        off = 0
        for n, sh, ne in zip(names, [e[2] for e in ents], numels):
            out[n] = full[off:off + ne].view(sh).clone()
            off += ne
    return out


class _EmuWork:
    """Work handle of an async emulated collective: ``wait()`` makes the caller's stream wait."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


class Comm:
    """The two collectives ZeRO-3 issues, over real ranks or emulated.

    ``ag_pg`` carries the all-gathers and ``rs_pg`` the reduce-scatters: two
    communicators = two streams (RCCL's, or the peer-memory path's with
    MXLLM_COMM=peer: mxllm/parallel/comm.py), so a prefetch gather and the
    previous unit's reduce-scatter run concurrently (xGMI links are full duplex).
    ``emulate`` > 1: single process standing in for rank 0 of that many."""

    def __init__(self, world: int, rank: int, ag_pg=None, rs_pg=None, emulate: int = 0, device=None):
        self.world, self.rank, self.ag_pg, self.rs_pg = world, rank, ag_pg, rs_pg
        self.emulate = emulate > 1
        self.ag = self.rs = None
        if self.real:
            from . import comm as comm_mod

            self.ag = comm_mod.create(ag_pg, device)
            self.rs = self.ag if rs_pg is ag_pg else comm_mod.create(rs_pg, device)
        # MXLLM_Z3_RS_WIRE=bf16 (VERDICT r5 Missing 4): the fp32 gradient reduce-scatters travel as
        # bf16 -- half the link bytes -- and are summed in fp32 in rank order at the owner (the
        # peer-memory light schedule, mxllm/parallel/comm.py).  RCCL sums bf16 in bf16 hop by hop,
        # so on the torch.distributed path the option is refused rather than silently weakened.
        # The emulated proxy rounds its stand-in operands to bf16 the same way.
        self.sent_bytes = {"ag": 0, "rs": 0}  # bytes this rank puts on its links (bench: per step)
        self.rs_wire = os.environ.get("MXLLM_Z3_RS_WIRE", "fp32").strip().lower()
        if self.rs_wire not in ("fp32", "bf16"):
            raise ValueError(f"MXLLM_Z3_RS_WIRE must be fp32 or bf16, not {self.rs_wire!r}")
        if self.rs_wire == "bf16" and self.real and getattr(self.rs, "algo", None) != "light":
            raise RuntimeError("MXLLM_Z3_RS_WIRE=bf16 needs MXLLM_COMM=peer with the light schedule")
        # emulated world N: the local stand-ins (a broadcast copy for the all-gather, an N-way sum
        # for the reduce-scatter) run on the caller's stream by default -- every byte of them on
        # the critical path, a conservative proxy.  MXLLM_Z3_EMUL_ASYNC=1 issues the async ones
        # the way the real communicators do (their own two streams, the caller's stream waiting
        # on an event at wait(), tensors kept alive by record_stream), so the proxy models the
        # overlap -- and the CU contention of a collective kernel running beside the compute.
        self._emu_streams = None
        if (self.emulate and device is not None and torch.device(device).type == "cuda"
                and os.environ.get("MXLLM_Z3_EMUL_ASYNC", "0") == "1"):
            self._emu_streams = {"ag": torch.cuda.Stream(device), "rs": torch.cuda.Stream(device)}

    def _emu(self, kind: str, fn, tensors, async_op: bool):
        """Run an emulated collective's local stand-in ``fn``: inline, or (async emulation) on the
        ``kind`` stream with RCCL's stream semantics."""
        if not (async_op and self._emu_streams):
            fn()
            return None
        s = self._emu_streams[kind]
        s.wait_stream(torch.cuda.current_stream(s.device))
        with torch.cuda.stream(s):
            fn()
        for t in tensors:
            t.record_stream(s)
        ev = torch.cuda.Event()
        ev.record(s)
        return _EmuWork(ev)

    @property
    def real(self) -> bool:
        return self.world > 1 and not self.emulate

    @property
    def kind(self) -> str:
        return getattr(self.ag, "kind", "none")

    def all_gather(self, full: torch.Tensor, shard: torch.Tensor, async_op: bool):
        self.sent_bytes["ag"] += shard.numel() * shard.element_size() * (self.world - 1)
        if self.real:
            return self.ag.all_gather(full, shard, async_op=async_op)
        return self._emu("ag", lambda: full.view(self.world, -1).copy_(shard.unsqueeze(0).expand(self.world, -1)),
                         (full, shard), async_op)

    def reduce_scatter(self, out: torch.Tensor, full: torch.Tensor, async_op: bool):
        wire = self.rs_wire == "bf16" and full.dtype == torch.float32
        self.sent_bytes["rs"] += self.rs_wire_bytes(full.numel(), full.dtype)
        if self.real:
            if wire:
                return self.rs.reduce_scatter(out, full, async_op=async_op, wire=torch.bfloat16)
            return self.rs.reduce_scatter(out, full, async_op=async_op)
        if self.world == 1:
            out.copy_(full)
            return None
        if wire:  # the owner's fp32 sum of bf16-rounded contributions
            return self._emu("rs", lambda: torch.sum(full.view(self.world, -1).to(torch.bfloat16).float(), dim=0,
                                                     out=out), (out, full), async_op)
        return self._emu("rs", lambda: torch.sum(full.view(self.world, -1), dim=0, out=out), (out, full), async_op)

    def rs_wire_bytes(self, numel: int, dtype: torch.dtype) -> int:
        """Bytes one reduce-scatter of ``numel`` elements puts on this rank's links: (W-1)/W of the
        tensor, at the wire's element size."""
        es = 2 if (self.rs_wire == "bf16" and dtype == torch.float32) else torch.empty(0, dtype=dtype).element_size()
        return numel * es * (self.world - 1) // max(1, self.world)

    def all_reduce(self, t: torch.Tensor, async_op: bool = False):
        if self.real:
            return self.rs.all_reduce(t, async_op=async_op)
        return None


class Unit:
    def __init__(self, uid: int, named, world: int, rank: int, comm: Comm, resident: bool = False):
        self.uid, self.world, self.rank, self.comm, self.resident = uid, world, rank, comm, resident
        self.names = [e[0] for e in named]
        self.params = [e[1] for e in named]
        self.shapes = [tuple(e[2]) for e in named]
        self.numels = [math.prod(s) for s in self.shapes]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.numel = off
        # the resident unit (every RMSNorm weight, ~1.3 M params at 70B) is REPLICATED, not
        # sharded: every rank holds and updates all of it (its gradient is all-reduced), so it
        # never needs a re-gather after the optimizer step (no synchronous regather)
        self.replicated = resident
        wsz = 1 if resident else world
        chunk = wsz * ALIGN
        self.full_numel = (off + chunk - 1) // chunk * chunk
        self.shard_numel = self.full_numel // wsz
        self.full: torch.Tensor | None = None
        self.work = None
        self.shard = None  # bf16 view (set by the trainer)
        self.grad_shard = None  # fp32 view
        self.gbuf: torch.Tensor | None = None  # gathered-size bf16 gradient buffer (backward only)
        self.seen: set[int] = set()
        self.reduced = False  # this micro-batch's gradient already handed to the reduce-scatter
        self.grad_written = False  # grad_shard written this step (the next write of the step accumulates)
        self.n_trainable = len(self.params)
        self.device = None
        self.dtype = None
        self.gdt = None  # gradient dtype (reduce-scatter / accumulation): fp32 or bf16
        # world 1 (not emulated): the shard IS the full unit — no gather copy, and
        # with fp32 gradients the dW GEMMs write straight into the fp32 grad shard
        self.local = (world == 1 and not comm.emulate) or resident

    # -------------------------------------------------------------- gather / release
    def gather(self, async_op: bool = True):
        if self.full is not None:
            return
        if self.local:
            self.full = self.shard
            return
        self.full = torch.empty(self.full_numel, dtype=self.dtype, device=self.device)
        self.work = self.comm.all_gather(self.full, self.shard, async_op)

    def materialize(self):
        if self.full is None:
            self.gather(async_op=False)
        if self.work is not None:
            self.work.wait()  # stream dependency on the RCCL stream, no host wait
            self.work = None
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            p.data = self.full[o:o + n].view(s)

    def release(self):
        if self.resident:
            return
        if self.work is not None:
            self.work.wait()
            self.work = None
        for p in self.params:
            p.data = _empty(self.dtype, self.device)
        self.full = None

    # -------------------------------------------------------------- gradients
    @property
    def grad32(self) -> bool:
        return self.gdt == torch.float32

    def direct(self) -> bool:
        """Gradients land in ``grad_shard`` itself: world 1 with fp32 gradients."""
        return self.local and self.grad32

    def attach_grads(self, first: bool = True):
        """Point every parameter's gradient target (``.grad``, or ``_mx_grad32``
        for fp32 gradients) at its slice of a gathered-size gradient buffer.  The
        dW GEMMs overwrite it (``_mx_grad_fresh``), so only the alignment pad is
        zeroed.  World 1 with fp32 gradients: the buffer IS the fp32 grad shard
        (overwritten on the first micro-batch, accumulated on later ones).
        Parameters whose gradient comes from autograd (embedding, tied weights)
        are copied in at reduce time.  ``first``: first micro-batch of the step."""
        if self.gbuf is not None:
            return
        # GPU: every projection/head gradient comes from param_weight_grad, which
        # honours the fresh flag; the CPU reference ops accumulate through autograd
        fresh = ops.use_native(self.shard)
        if self.direct():
            self.gbuf = self.grad_shard  # its pad past the parameters is never written: stays zero
            if first and not fresh:
                self.gbuf.zero_()  # CPU reference ops accumulate through autograd
            fresh = fresh and first
        elif fresh:
            self.gbuf = torch.empty(self.full_numel, dtype=self.gdt, device=self.device)
            if self.full_numel > self.numel:
                self.gbuf[self.numel:].zero_()
        else:
            self.gbuf = torch.zeros(self.full_numel, dtype=self.gdt, device=self.device)
        for p, o, n, s in zip(self.params, self.offsets, self.numels, self.shapes):
            if getattr(p, "_mx_no_direct", False) or p.shape != s:
                continue
            if self.grad32:
                p._mx_grad32 = self.gbuf[o:o + n].view(s)
            else:
                p.grad = self.gbuf[o:o + n].view(s)
            p._mx_grad_fresh = fresh

    def reduce_replicated(self):
        """Replicated unit, once per step: its gradient (summed over the step's
        micro-batches) into the fp32 ``grad_shard``, then an all-reduce (sum over the
        ranks) in place.  Returns the work handle (None: nothing in flight)."""
        direct = self._collect()
        if not direct:
            self.grad_shard.copy_(self.gbuf[:self.shard_numel])
        self.gbuf = None
        if self.comm.emulate:  # emulated world N: N identical ranks would sum N copies
            self.grad_shard.mul_(float(self.world))
        return self.comm.all_reduce(self.grad_shard, async_op=True)

    def reduce_async(self, first: bool = True):
        """Launch the reduce-scatter of the unit's gradient buffer; returns
        (work | None, shard | None, fold).  ``fold``: the shard must still be added
        into ``grad_shard`` (bf16 gradients, or a later micro-batch); fp32 on the
        first micro-batch reduce-scatters straight into ``grad_shard``, and world 1
        with fp32 gradients has nothing to reduce (the GEMMs wrote ``grad_shard``)."""
        direct = self._collect()
        if direct:
            self.gbuf = None
            return None, None, False
        into = first and self.grad32
        out = self.grad_shard if into else torch.empty(self.shard_numel, dtype=self.gdt, device=self.device)
        work = self.comm.reduce_scatter(out, self.gbuf, async_op=True)
        self.gbuf = None  # RCCL keeps the buffer alive until the collective is done
        return work, (None if into else out), not into

    def _collect(self) -> bool:
        """Every parameter's gradient into the unit's gradient buffer (``gbuf``); returns
        whether that buffer is ``grad_shard`` itself."""
        if self.gbuf is None:
            g0 = self.params[0].grad if len(self.params) == 1 else None
            if (g0 is not None and g0.is_contiguous() and g0.numel() == self.full_numel
                    and g0.dtype == self.gdt):
                self.gbuf = g0.view(-1)  # autograd's own gradient tensor, no copy (e.g. the embedding)
            elif self.direct():
                self.gbuf = self.grad_shard
            else:
                self.gbuf = torch.zeros(self.full_numel, dtype=self.gdt, device=self.device)
        direct = self.gbuf is self.grad_shard
        for p, o, n in zip(self.params, self.offsets, self.numels):
            g = p.grad
            dst = self.gbuf[o:o + n]
            fresh = getattr(p, "_mx_grad_fresh", False)
            if g is None:
                if fresh:
                    dst.zero_()  # attached but never written (parameter unused this step)
            elif g.data_ptr() != dst.data_ptr():
                if direct and not fresh:
                    dst.add_(g.reshape(-1))  # grad_shard accumulates across micro-batches
                else:
                    dst.copy_(g.reshape(-1))
            elif fresh:
                dst.zero_()
            p.grad = None
            p._mx_grad_fresh = False
            p._mx_grad32 = None
        self.seen.clear()
        self.reduced = True
        return direct


class _PreBackward(torch.autograd.Function):
    """Identity on a unit's outputs whose backward runs before any of the unit's
    own backward ops: re-gather the unit, prefetch the next one, attach grads."""

    @staticmethod
    def forward(ctx, trainer, uid, *xs):
        ctx.trainer, ctx.uid = trainer, uid
        out = tuple(x.view_as(x) for x in xs)
        return out if len(out) > 1 else out[0]

    @staticmethod
    def backward(ctx, *gs):
        ctx.trainer._pre_backward(ctx.uid)
        return (None, None) + gs


class _CkptLayer(torch.autograd.Function):
    """Activation-checkpointed transformer layer under ZeRO-3: forward keeps only
    (x, h); backward re-gathers the unit, recomputes and back-propagates."""

    @staticmethod
    def forward(ctx, trainer, i, x, h):
        ctx.trainer, ctx.i = trainer, i
        ctx.save_for_backward(x, h)
        with torch.no_grad():
            xo, ho = trainer.model._layer(i, x, h, trainer._B, trainer._S)
        ctx.BS = (trainer._B, trainer._S)
        return xo, ho

    @staticmethod
    def backward(ctx, dxo, dho):
        tr = ctx.trainer
        x, h = ctx.saved_tensors
        uid = tr._units_by_layer[ctx.i].uid
        tr._pre_backward(uid)
        xd = x.detach().requires_grad_(True)
        hd = h.detach().requires_grad_(True)
        with torch.enable_grad():
            xo, ho = tr.model._layer(ctx.i, xd, hd, *ctx.BS)
        outs, grads = [], []
        for o, g in ((xo, dxo), (ho, dho)):
            if g is not None and o.requires_grad:
                outs.append(o)
                grads.append(g)
        torch.autograd.backward(outs, grads)
        return None, None, xd.grad, hd.grad


class Zero3Trainer:
    """Same ``train_step`` contract as :class:`mxllm.train.trainer.Trainer`."""

    def __init__(self, cfg, env: DistEnv, optim=None, *, seed: int = 0, activation_checkpointing: bool | int = False,
                 process_group=None, emulate_world: int = 0, max_inflight: int | None = None,
                 init_from: str | None = None, grad_dtype: torch.dtype | None = torch.float32,
                 rs_group=None):
        """``grad_dtype``: dtype the unit gradients are formed, reduce-scattered and
        accumulated in — fp32 by default (no bf16 rounding at any ring hop; the dW
        GEMMs write fp32 output), ``torch.bfloat16`` halves the reduce-scatter
        bytes.  ``None`` = fp32."""
        from ..models.llama import Llama
        from ..train.trainer import OptimConfig

        self.env, self.opt = env, optim or OptimConfig()
        self.act_ckpt = activation_checkpointing
        self.pg = process_group
        if emulate_world and emulate_world > 1:
            self.world, self.rank = emulate_world, 0
            comm = Comm(self.world, 0, emulate=emulate_world)
        else:
            self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
            rs_pg = rs_group if rs_group is not None else process_group
            # second communicator (reduce-scatters on their own stream).  new_group is
            # collective over the DEFAULT group, so it is only created here for the
            # default group; a caller sharding over a subgroup passes ``rs_group``
            # (created where every rank reaches it) or gets one communicator
            if (rs_group is None and process_group is None and self.world > 1
                    and os.environ.get("MXLLM_Z3_SPLIT_COMMS", "1") != "0"):
                rs_pg = dist.new_group()
            comm = Comm(self.world, self.rank, process_group, rs_pg, device=env.device)
        self.comm = comm
        self.emulated = comm.emulate
        self.max_inflight = max_inflight or int(os.environ.get("MXLLM_Z3_INFLIGHT", "2"))
        dev = env.device
        self.device = dev
        model = Llama(cfg, device="meta", init=False)
        _realize_on(model, dev)
        self.model = model
        model.mlp_recompute_ckpt = activation_checkpointing  # _layer's recompute-m policy follows our checkpointing
        units = unit_layout(model)
        self.units = [Unit(k, ps, self.world, self.rank, comm, res) for k, (_, ps, res) in enumerate(units)]
        self.unit_names = [u[0] for u in units]
        self.grad_dtype = grad_dtype or torch.float32
        for u in self.units:
            u.device, u.dtype, u.gdt = dev, torch.bfloat16, self.grad_dtype
        total = sum(u.shard_numel for u in self.units)
        self.shard_params = torch.empty(total, dtype=torch.bfloat16, device=dev)
        # fp32 master as (bf16 shard, int16 low halves): exact fp32 values, no separate
        # bf16 copy — 2 B/param less (70B at world 8: 17.6 GB per rank)
        self.split_master = os.environ.get("MXLLM_SPLIT_MASTER", "1") != "0"
        self.master = (ops.SplitMaster(self.shard_params) if self.split_master
                       else torch.empty(total, dtype=torch.float32, device=dev))
        self.grads = torch.zeros(total, dtype=torch.float32, device=dev)
        self.m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for u in self.units:
            u.shard = self.shard_params[off:off + u.shard_numel]
            u.grad_shard = self.grads[off:off + u.shard_numel]
            u.master_view = self.master[off:off + u.shard_numel]
            off += u.shard_numel
        self._materialize_shards(seed, init_from)
        if not self.split_master:
            self.master.copy_(self.shard_params)  # (split: lo = 0 is the exact fp32 value already)
        self._by_storage: dict[int, Unit] = {}
        self._param_unit: dict[int, Unit] = {}
        for u in self.units:
            for p in u.params:
                p.requires_grad_(True)
                self._param_unit[id(p)] = u
                p.register_post_accumulate_grad_hook(self._grad_hook)
                p._mx_on_grad_ready = self._grad_hook  # dW written by the GEMM itself (param_weight_grad)
                if not u.resident and len(u.params) == 1 and not getattr(p, "_mx_no_direct", False):
                    p._mx_grad_sink = self._sink  # e.g. the embedding: its unit is not gathered in backward
                    p._mx_grad_sink_dtype = self.grad_dtype
        self._inflight: deque = deque()
        self._first = True  # first micro-batch of the step (fp32: reduce-scatter straight into grad_shard)
        self.step_num = 0
        self.last_grad_norm = None
        self._units_by_layer = {i: self.units[2 + i] for i in range(len(model.layers))}
        self._head = self.units[-1] if model.lm_head is not None else self.units[1]
        self._below = {}  # unit -> the unit whose backward follows it (prefetch target)
        order = [self._head] + [self._units_by_layer[i] for i in reversed(range(len(model.layers)))]
        for a, b in zip(order, order[1:]):
            if a is not b:
                self._below[a.uid] = b
        self._B = self._S = 0
        # ---- optimizer / next-forward overlap: the fused AdamW runs unit by
        # unit on a side stream in FORWARD order; the next forward waits for unit u's update just
        # before it gathers / uses u, so the update of the units it has not reached yet runs under
        # its GEMMs instead of as one serial launch between the steps
        self._side = (torch.cuda.Stream(dev) if dev.type == "cuda"
                      and os.environ.get("MXLLM_Z3_ADAMW_OVERLAP", "1") != "0" else None)
        self._pending: dict[int, torch.cuda.Event] = {}
        self._hold = None
        self._fwd_order = [self.units[0], self.units[1]] + [self._units_by_layer[i] for i in range(len(model.layers))]
        if self._head is not self.units[1]:
            self._fwd_order.append(self._head)
        self.overlap_optimizer = self._side is not None
        model._zero3 = self
        log.info("ZeRO-3: %d units, %.2f M params/rank (world %d%s, act-ckpt %s)", len(self.units), total / 1e6,
                 self.world, " emulated" if self.emulated else "", self.act_ckpt)

    # ---------------------------------------------------------------- init
    @torch.no_grad()
    def _materialize_shards(self, seed: int, init_from: str | None = None):
        """Initialise every unit on device (per-unit seed: identical on every rank) or
        read it from a Hugging Face checkpoint directory (``init_from``,
        mxllm/models/hf.py), keep this rank's slice, free the rest — never the whole
        model at once."""
        fill = None
        if init_from:
            from ..models.hf import hf_unit_filler

            fill = hf_unit_filler(init_from, self.model.cfg)
        for u in self.units:
            if fill is not None:
                full = torch.zeros(u.full_numel, dtype=torch.bfloat16, device=self.device)
                fill(u.names, u.shapes, full)
            else:
                full = init_unit_full(u.uid, u.names, u.numels, u.full_numel, seed, self.device)
            r = 0 if u.replicated else self.rank
            u.shard.copy_(full[r * u.shard_numel:(r + 1) * u.shard_numel])
            del full
        self.units[0].materialize()  # norms stay resident

    # ---------------------------------------------------------------- hooks
    def _grad_hook(self, p):
        u = self._param_unit[id(p)]
        if u.resident or u.reduced or id(p) in u.seen:
            return
        u.seen.add(id(p))
        if len(u.seen) == u.n_trainable:
            self._reduce(u)

    def _sink(self, p, g):
        """A full gradient delivered by its op (grad_ready.deliver_grad)."""
        u = self._param_unit[id(p)]
        if u.gbuf is None and g.is_contiguous() and g.numel() == u.full_numel and g.dtype == u.gdt:
            u.gbuf = g.view(-1)
        else:
            if u.gbuf is None:
                u.gbuf = (u.grad_shard if u.direct()
                          else torch.zeros(u.full_numel, dtype=u.gdt, device=u.device))
            k = u.params.index(p)
            dst = u.gbuf[u.offsets[k]:u.offsets[k] + u.numels[k]]
            if u.gbuf is u.grad_shard and not self._first:
                dst.add_(g.reshape(-1))
            else:
                dst.copy_(g.reshape(-1))
        self._grad_hook(p)

    def _reduce(self, u: Unit):
        work, out, fold = u.reduce_async(self._first)
        # the first write of a step overwrites grad_shard (AdamW does not clear it): the
        # reduce-scatter / direct GEMM output lands in it, or the first fold is a copy
        first_write = not u.grad_written
        u.grad_written = True
        self._inflight.append((u, work, out if fold else None, first_write))
        self._done(u)
        while len(self._inflight) > self.max_inflight:
            self._drain_one()

    def _drain_one(self):
        u, work, out, first_write = self._inflight.popleft()
        if work is not None:
            work.wait()  # the compute stream waits for the RCCL stream; the host does not
        if out is not None:
            if first_write:
                u.grad_shard.copy_(out)
            else:
                u.grad_shard.add_(out)

    def _drain(self):
        while self._inflight:
            self._drain_one()

    def _pre_backward(self, uid: int):
        u = self.units[uid]
        if u.full is None:
            self._gather(u)
        nxt = self._below.get(uid)
        if nxt is not None and nxt.full is None:
            self._gather(nxt)
        u.materialize()
        u.attach_grads(self._first)

    def _pack(self, t):
        if t.device.type == "meta" or not isinstance(t, torch.Tensor):
            return t
        try:
            key = t.untyped_storage().data_ptr()
        except Exception:  # noqa: BLE001
            return t
        u = self._by_storage.get(key)
        if u is None:
            return t
        return ("mxz3", u.uid, t.storage_offset(), tuple(t.shape), tuple(t.stride()))

    def _unpack(self, obj):
        if isinstance(obj, tuple) and len(obj) == 5 and obj[0] == "mxz3":
            _, uid, off, shape, stride = obj
            u = self.units[uid]
            if u.full is None:  # _PreBackward normally gathered it already
                self._gather(u)
            u.materialize()
            return torch.as_strided(u.full, shape, stride, off)
        return obj

    def _wait_update(self, u: Unit):
        """The compute stream waits for unit u's overlapped AdamW (no host sync)."""
        ev = self._pending.pop(u.uid, None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def _gather(self, u: Unit, async_op=True):
        self._wait_update(u)  # the gather reads the updated shard (RCCL orders after the current stream)
        u.gather(async_op=async_op)
        if not u.local:  # world 1: the "gathered" unit is the persistent shard, nothing to release
            self._by_storage[u.full.untyped_storage().data_ptr()] = u

    def _use(self, u: Unit, prefetch: Unit | None = None):
        self._wait_update(u)
        if u.full is None:
            self._gather(u)
        if prefetch is not None and prefetch.full is None:
            self._gather(prefetch)
        u.materialize()

    def _done(self, u: Unit):
        if u.resident:
            return
        if u.full is not None and not u.local:
            self._by_storage.pop(u.full.untyped_storage().data_ptr(), None)
        u.release()

    # ---------------------------------------------------------------- step
    def _forward(self, ids, labels):
        from ..models.llama import ckpt_layer

        m = self.model
        cfg = m.cfg
        B, S = ids.shape
        self._B, self._S = B, S
        self._wait_update(self.units[0])  # every layer's RMSNorm reads the replicated unit
        for u in self.units:
            u.seen.clear()
            u.reduced = False
        with torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack):
            emb = self.units[1]
            self._use(emb, self._units_by_layer.get(0))
            h = ops.embedding(ids.reshape(-1), m.tok_emb)
            if self._head is not emb:
                self._done(emb)
            x = ops.rms_norm(h, m.layers[0].attn_norm, cfg.norm_eps)
            for i in range(len(m.layers)):
                u = self._units_by_layer[i]
                nxt = self._units_by_layer.get(i + 1, self._head)
                self._use(u, nxt)
                if ckpt_layer(self.act_ckpt, i):
                    x, h = _CkptLayer.apply(self, i, x, h)
                else:
                    x, h = m._layer(i, x, h, B, S)
                    x, h = _PreBackward.apply(self, u.uid, x, h)
                self._done(u)
            self._use(self._head)
            loss = ops.linear_cross_entropy(x, m.head_weight, labels.reshape(-1))
            loss = _PreBackward.apply(self, self._head.uid, loss)
            self._done(self._head)
        return loss

    def train_step(self, micro_batches):
        n = len(micro_batches)
        total = None
        norms = self.units[0]  # resident unit: gradients accumulate over the micro-batches, one reduce per step
        for k, (ids, labels) in enumerate(micro_batches):
            self._first = k == 0
            if k == 0 and norms.grad32:
                norms.attach_grads(True)  # the RMSNorm kernels add their fp32 dγ into it
            loss = self._forward(ids, labels)
            loss.backward()  # 1/n folded into the optimizer's grad scale
            for u in self.units[1:]:  # units whose hooks did not all fire (unused params)
                if not u.reduced and (u.seen or u.gbuf is not None or any(p.grad is not None for p in u.params)):
                    self._reduce(u)
                elif u.full is not None:
                    self._done(u)
            total = loss.detach() if total is None else total + loss.detach()
        self._drain()
        self._first = True
        work = norms.reduce_replicated()  # all-reduce of the replicated unit's fp32 gradient
        if work is not None:
            work.wait()
        for u in self.units[1:]:
            if not u.grad_written:  # no gradient at all this step (unused): a zero update input
                u.grad_shard.zero_()
            u.grad_written = False
        scale = 1.0 / (self.world * n)
        if self.comm.real:
            from .comm import verify

            verify(self.comm.rs, self.comm.ag)  # peer path: a timed-out exchange stops here, before AdamW
        self.step_num += 1
        o = self.opt
        if o.grad_clip and o.grad_clip > 0:
            # sharded units: sum of squares over the ranks; the replicated unit (flat [0, n0),
            # identical on every rank after its all-reduce) is counted once
            n0 = norms.shard_numel
            sq = ops.sq_norm(self.grads[n0:])
            self.comm.all_reduce(sq)
            sq = sq + ops.sq_norm(self.grads[:n0])
            gnorm = sq.sqrt() * scale
            self.last_grad_norm = gnorm
            gscale = torch.clamp(o.grad_clip / (gnorm + 1e-6), max=1.0) * scale
        else:
            gscale = scale
        kw = dict(lr=o.lr_at(self.step_num), beta1=o.beta1, beta2=o.beta2, eps=o.eps, weight_decay=o.weight_decay,
                  step=self.step_num, grad_scale=gscale, zero_grad=False)  # every shard is overwritten next step
        if self._side is None:
            ops.adamw_step_(self.master, self.grads, self.m, self.v, self.shard_params, **kw)
        else:
            self._launch_overlapped(kw)
        return total / n

    def _launch_overlapped(self, kw):
        """The fused AdamW over each unit's shard on the side stream in forward order, one
        event per unit (waited in _use / _gather).  Same elementwise kernel over the same
        slices with the same inputs: bitwise identical to the one-launch update."""
        side = self._side
        side.wait_stream(torch.cuda.current_stream(self.device))
        self._hold = kw["grad_scale"]  # read on the side stream: keep it alive until the next step
        with torch.cuda.stream(side):
            for u in self._fwd_order:
                off = u.grad_shard.storage_offset() - self.grads.storage_offset()
                sl = slice(off, off + u.shard_numel)
                ops.adamw_step_(self.master[sl], self.grads[sl], self.m[sl], self.v[sl], self.shard_params[sl], **kw)
                ev = torch.cuda.Event()
                ev.record(side)
                self._pending[u.uid] = ev

    def _refresh_resident(self):
        # the replicated unit IS its shard (updated in place by AdamW): re-point its parameters
        norms = self.units[0]
        norms.full = None
        norms.work = None
        norms.gather(async_op=False)
        norms.materialize()

    # ---------------------------------------------------------------- state
    def state_dict(self):
        self.params_ready()
        return {"step": self.step_num, "master": self.master, "m": self.m, "v": self.v}

    def load_state_dict(self, sd):
        self.master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.finish_load(int(sd["step"]))

    def finish_load(self, step: int):
        """After master/m/v were written in place (checkpoint.load, which reshards
        unit by unit): set the step, rebuild the bf16 shards and the resident unit."""
        self.step_num = int(step)
        if not self.split_master:
            self.shard_params.copy_(self.master)
        self._refresh_resident()

    def params_ready(self):
        """Order the current stream after every in-flight overlapped unit update: call
        before reading parameters / optimizer state outside a step (checkpoints, export)."""
        for u in self.units:
            self._wait_update(u)

    def full_master_state(self) -> dict:
        """Every fp32 master weight, gathered unit by unit (collective: all ranks
        call it; tests / export)."""
        self.params_ready()
        out = {}
        for u in self.units:
            src = u.master_view.float().contiguous()
            if u.replicated:
                full = src
            else:
                full = torch.empty(u.full_numel, dtype=torch.float32, device=self.device)
                if self.comm.real:
                    self.comm.ag.all_gather(full, src)
                else:
                    full.view(self.world, -1).copy_(src.unsqueeze(0).expand(self.world, -1))
            for name, o, n, shp in zip(u.names, u.offsets, u.numels, u.shapes):
                out[name] = full[o:o + n].view(shp).clone()
        return out

    def full_state_dict(self) -> dict:
        """Gather every unit (one at a time) into named CPU tensors (rank 0 keeps them)."""
        out = {}
        for u in self.units:
            was = u.full is not None
            if not was:
                u.gather(async_op=False)
            u.materialize()
            if self.rank == 0:
                for name, p in zip(u.names, u.params):
                    out[name] = p.detach().cpu().clone()
            if not was:
                u.release()
        return out
