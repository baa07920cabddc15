"""ZeRO-3 / fully-sharded data parallel for full fine-tuning.

Llama-3.1-70B full fine-tuning needs 16 B/param = 1,129 GB of state: it only
fits an 8 x 288 GB MI355X node sharded.  Design:

  * units: the model is cut into flat parameter units — the embedding, each
    transformer layer's four projection matrices, the LM head — plus one small
    always-resident unit holding every RMSNorm weight.  Each unit is a flat
    bf16 buffer split evenly over the ranks; a rank keeps only its slice
    (bf16 compute shard + fp32 master + Adam m, v + fp32 grad shard), all as
    views into ONE flat per-rank buffer each, so the optimizer is one fused
    AdamW launch per step.
  * forward: a unit is all-gathered (``all_gather_into_tensor`` over RCCL /
    xGMI: each rank receives 7/8 of a 1.7 GB layer) just before use, with the
    NEXT unit's gather already in flight (async), and released after use;
  * autograd never keeps a gathered weight alive: a ``saved_tensors_hooks``
    pair saves a (unit, offset, shape, stride) handle instead of any tensor
    that lives in a gathered buffer, and re-gathers the unit on unpack during
    backward (prefetching the unit below it);
  * gradients: when the last parameter of a unit has accumulated its gradient
    (post-accumulate-grad hooks), the unit's full gradient is reduce-scattered
    into the rank's fp32 grad shard and the gathered weights are freed.
  * the model is built on the meta device and materialised unit by unit with
    a per-unit seed, so no rank ever holds the full 141 GB model.
Reference parity: none — the reference advertises 70B fine-tuning
(README.md:1-3) with no training code.
"""
from __future__ import annotations

import logging
import math

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


class Unit:
    def __init__(self, uid: int, named, world: int, rank: int, pg, resident: bool = False):
        self.uid, self.world, self.rank, self.pg, self.resident = uid, world, rank, pg, resident
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
        chunk = world * ALIGN
        self.full_numel = (off + chunk - 1) // chunk * chunk
        self.shard_numel = self.full_numel // world
        self.full: torch.Tensor | None = None
        self.work = None
        self.shard = None  # bf16 view (set by the trainer)
        self.grad_shard = None  # fp32 view
        self.pending = 0
        self.device = None
        self.dtype = None

    # -------------------------------------------------------------- gather / release
    def gather(self, async_op: bool = True):
        if self.full is not None:
            return
        self.full = torch.empty(self.full_numel, dtype=self.dtype, device=self.device)
        if self.world > 1:
            self.work = dist.all_gather_into_tensor(self.full, self.shard, group=self.pg, async_op=async_op)
        else:
            self.full.copy_(self.shard)

    def materialize(self):
        if self.full is None:
            self.gather(async_op=False)
        if self.work is not None:
            self.work.wait()
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
    def reduce_grads(self, accumulate: bool):
        parts = []
        for p, n in zip(self.params, self.numels):
            g = p.grad
            parts.append(g.reshape(-1).to(self.dtype) if g is not None else torch.zeros(n, dtype=self.dtype,
                                                                                         device=self.device))
            p.grad = None
        pad = self.full_numel - self.numel
        if pad:
            parts.append(torch.zeros(pad, dtype=self.dtype, device=self.device))
        gfull = torch.cat(parts)
        out = torch.empty(self.shard_numel, dtype=self.dtype, device=self.device)
        if self.world > 1:
            dist.reduce_scatter_tensor(out, gfull, op=dist.ReduceOp.SUM, group=self.pg)
        else:
            out.copy_(gfull)
        if accumulate:
            self.grad_shard.add_(out.float())
        else:
            self.grad_shard.copy_(out)


class Zero3Trainer:
    """Same ``train_step`` contract as :class:`mxllm.train.trainer.Trainer`."""

    def __init__(self, cfg, env: DistEnv, optim=None, *, seed: int = 0, activation_checkpointing: bool = False,
                 process_group=None):
        from ..models.llama import Llama
        from ..train.trainer import OptimConfig

        if activation_checkpointing:
            raise NotImplementedError("ZeRO-3 + activation checkpointing is not supported yet")
        self.env, self.opt = env, optim or OptimConfig()
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        dev = env.device
        self.device = dev
        model = Llama(cfg, device="meta", init=False)
        _realize_on(model, dev)
        self.model = model
        units = unit_layout(model)
        self.units = [Unit(k, ps, self.world, self.rank, self.pg, res) for k, (_, ps, res) in enumerate(units)]
        self.unit_names = [u[0] for u in units]
        for u in self.units:
            u.device, u.dtype = dev, torch.bfloat16
        total = sum(u.shard_numel for u in self.units)
        self.shard_params = torch.empty(total, dtype=torch.bfloat16, device=dev)
        self.master = torch.empty(total, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(total, dtype=torch.float32, device=dev)
        self.m = torch.zeros(total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for u in self.units:
            u.shard = self.shard_params[off:off + u.shard_numel]
            u.grad_shard = self.grads[off:off + u.shard_numel]
            u.master_view = self.master[off:off + u.shard_numel]
            off += u.shard_numel
        self._materialize_shards(seed)
        self.master.copy_(self.shard_params)
        self._by_storage: dict[int, Unit] = {}
        self._param_unit: dict[int, Unit] = {}
        for u in self.units:
            for p in u.params:
                p.requires_grad_(True)
                self._param_unit[id(p)] = u
                p.register_post_accumulate_grad_hook(self._grad_hook)
                if not u.resident:  # gradient about to be accumulated: the unit must be materialised
                    p.register_hook(self._make_pre_grad_hook(u))
        self._accumulate = False
        self.step_num = 0
        self.last_grad_norm = None
        self._units_by_layer = {i: self.units[2 + i] for i in range(len(model.layers))}
        self._head = self.units[-1] if model.lm_head is not None else self.units[1]
        model._zero3 = self
        log.info("ZeRO-3: %d units, %.2f M params/rank (world %d)", len(self.units), total / 1e6, self.world)

    # ---------------------------------------------------------------- init
    @torch.no_grad()
    def _materialize_shards(self, seed: int):
        """Initialise every unit on device (per-unit seed: identical on every rank),
        keep this rank's slice, free the rest — never the whole model at once."""
        for u in self.units:
            full = init_unit_full(u.uid, u.names, u.numels, u.full_numel, seed, self.device)
            u.shard.copy_(full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel])
            del full
        self.units[0].materialize()  # norms stay resident

    # ---------------------------------------------------------------- hooks
    def _make_pre_grad_hook(self, u):
        def hook(g):
            if u.full is None:
                self._gather(u, async_op=False)
            u.materialize()
            return g
        return hook

    def _grad_hook(self, p):
        u = self._param_unit[id(p)]
        u.pending -= 1
        if u.pending == 0 and not u.resident:
            u.reduce_grads(self._accumulate)
            self._done(u)

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
            if u.full is None:
                self._gather(u)
                self._prefetch_below(u)
            u.materialize()
            return torch.as_strided(u.full, shape, stride, off)
        return obj

    def _gather(self, u: Unit, async_op=True):
        u.gather(async_op=async_op)
        self._by_storage[u.full.untyped_storage().data_ptr()] = u

    def _prefetch_below(self, u: Unit):
        if 2 < u.uid < len(self.units):
            nxt = self.units[u.uid - 1]
            if nxt.full is None:
                self._gather(nxt)

    def _use(self, u: Unit, prefetch: Unit | None = None):
        if u.full is None:
            self._gather(u)
        if prefetch is not None and prefetch.full is None:
            self._gather(prefetch)
        u.materialize()

    def _done(self, u: Unit):
        if u.full is not None:
            self._by_storage.pop(u.full.untyped_storage().data_ptr(), None)
        u.release()

    # ---------------------------------------------------------------- step
    def _forward(self, ids, labels):
        m = self.model
        cfg = m.cfg
        B, S = ids.shape
        for u in self.units:
            u.pending = sum(1 for p in u.params if p.requires_grad)
        with torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack):
            emb = self.units[1]
            self._use(emb, self._units_by_layer.get(0))
            h = ops.embedding(ids.reshape(-1), m.tok_emb)
            if not self._head is emb:
                self._done(emb)
            x = ops.rms_norm(h, m.layers[0].attn_norm, cfg.norm_eps)
            for i in range(len(m.layers)):
                u = self._units_by_layer[i]
                nxt = self._units_by_layer.get(i + 1, self._head)
                self._use(u, nxt)
                x, h = m._layer(i, x, h, B, S)
                self._done(u)
            self._use(self._head)
            loss = ops.linear_cross_entropy(x, m.head_weight, labels.reshape(-1))
            self._done(self._head)
        return loss

    def train_step(self, micro_batches):
        n = len(micro_batches)
        total = None
        for i, (ids, labels) in enumerate(micro_batches):
            self._accumulate = i > 0
            loss = self._forward(ids, labels)
            (loss / n if n > 1 else loss).backward()
            total = loss.detach() if total is None else total + loss.detach()
        # resident unit (norms): all-reduce-scatter its grads now
        norms = self.units[0]
        norms.reduce_grads(accumulate=False)
        for u in self.units[1:]:  # any unit whose hooks did not all fire (unused params)
            if any(p.grad is not None for p in u.params):
                u.reduce_grads(accumulate=True)
            if u.full is not None:
                self._done(u)
        scale = 1.0 / (self.world * n)
        self.step_num += 1
        o = self.opt
        if o.grad_clip and o.grad_clip > 0:
            sq = ops.sq_norm(self.grads)
            if self.world > 1:
                dist.all_reduce(sq, group=self.pg)
            gnorm = sq.sqrt() * scale
            self.last_grad_norm = gnorm
            gscale = torch.clamp(o.grad_clip / (gnorm + 1e-6), max=1.0) * scale
        else:
            gscale = scale
        ops.adamw_step_(self.master, self.grads, self.m, self.v, self.shard_params, lr=o.lr_at(self.step_num),
                        beta1=o.beta1, beta2=o.beta2, eps=o.eps, weight_decay=o.weight_decay, step=self.step_num,
                        grad_scale=gscale, zero_grad=True)  # shard grads cleared in the same pass
        self._refresh_resident()
        return total / n

    def _refresh_resident(self):
        # the resident unit's gathered copy must follow its updated shards
        norms = self.units[0]
        norms.full = None
        norms.work = None
        norms.gather(async_op=False)
        norms.materialize()

    # ---------------------------------------------------------------- state
    def state_dict(self):
        return {"step": self.step_num, "master": self.master, "m": self.m, "v": self.v}

    def load_state_dict(self, sd):
        self.step_num = int(sd["step"])
        self.master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.shard_params.copy_(self.master)
        self._refresh_resident()

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
