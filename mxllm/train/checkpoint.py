"""Checkpoint / resume — safetensors + JSON manifest, streamed.

Layout ``<dir>/step_<N>/`` (format 2):
  manifest.json                 step, world, parallel kind, flat-buffer slot table
                                / ZeRO-3 unit table, piece list, loader state
  optim/part_<k>.safetensors    DDP: rank 0's optimizer state (fp32 master, m, v)
                                in flat-buffer ranges of <= PIECE_ELEMS elements
  rank_<r>.safetensors          ZeRO-1: rank r's optimizer shards (compact layout)
  z3/rank_<r>/unit_<u>.safetensors
                                ZeRO-3: rank r's shard of unit u (master, m, v)
  model/part_<k>.safetensors    trainable weights by name (DDP / ZeRO-1: rank 0, after
                                every in-flight update landed), loadable by
                                ``load_model_weights`` for serving / export
``<dir>/latest`` holds the newest complete step (written last = atomic commit).

Streaming: no step ever stages more than one piece / one unit shard on the host
(``staged_peak_bytes``), so a 70B ZeRO-3 rank (~106 GB of fp32 state) never
builds a whole-state dict.  Resharding: a ZeRO-3 checkpoint written at world N
resumes at world M — every rank reads the byte ranges of its new shard out of
the old ranks' unit files (``safe_open(...).get_slice``, nothing else is read).
A DDP checkpoint resumes into a different flat layout by slot name.
Only safetensors/JSON are used: nothing is ever unpickled.
"""
from __future__ import annotations

import json
import logging
import os
import shutil

import torch
import torch.distributed as dist
from safetensors import safe_open
from safetensors.torch import load_file, save_file

log = logging.getLogger("mxllm.ckpt")
FORMAT = 2
PIECE_ELEMS = int(os.environ.get("MXLLM_CKPT_PIECE_ELEMS", str(64 << 20)))  # x (master, m, v) x 4 B = 768 MB
_STAGED = {"peak": 0}


def staged_peak_bytes() -> int:
    """Largest host staging of one checkpoint write so far (bytes)."""
    return _STAGED["peak"]


def _rank_world():
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _barrier():
    if dist.is_initialized():
        from ..parallel import runtime

        runtime.barrier()


def _write(path: str, tensors: dict):
    """Stage ``tensors`` on the host and write one safetensors file."""
    host = {k: v.detach().contiguous().cpu() for k, v in tensors.items()}
    _STAGED["peak"] = max(_STAGED["peak"], sum(t.numel() * t.element_size() for t in host.values()))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    save_file(host, path)
    del host


def _kind(trainer) -> str:
    if hasattr(trainer, "units"):
        return "zero3"
    return "zero1" if getattr(trainer, "zero1", None) is not None else "ddp"


def save(ckpt_dir: str, trainer, step: int, extra: dict | None = None, sharded: bool | None = None,
         keep: int = 2) -> str:
    """Collective: every rank calls it.  ``sharded`` is accepted for API
    compatibility; what each rank writes follows from the trainer (DDP: rank 0,
    ZeRO-1 / ZeRO-3: every rank its own shards)."""
    del sharded
    rank, world = _rank_world()
    d = os.path.join(ckpt_dir, f"step_{step}")
    if rank == 0:
        os.makedirs(d, exist_ok=True)
    _barrier()
    if hasattr(trainer, "params_ready"):
        trainer.params_ready()  # overlapped optimizer chunks / ZeRO-1 gathers have landed
    kind = _kind(trainer)
    man = {"format": FORMAT, "step": step, "world_size": world, "kind": kind, "extra": extra or {}}
    if kind == "zero3":
        man["units"] = _save_zero3(d, trainer, rank)
    elif kind == "zero1":
        _write(os.path.join(d, f"rank_{rank}.safetensors"),
               {"master": trainer._master, "m": trainer.m, "v": trainer.v})
    elif rank == 0:
        man["pieces"] = _save_flat(d, trainer)
    if kind != "zero3":
        man["layout"] = trainer.flat.state_dict()
        if rank == 0:
            man["model_parts"] = _save_model(d, trainer.model)
    if rank == 0:
        with open(os.path.join(d, "manifest.json"), "w") as f:
            json.dump(man, f, indent=1)
    _barrier()
    if rank == 0:
        with open(os.path.join(ckpt_dir, "latest.tmp"), "w") as f:
            f.write(str(step))
        os.replace(os.path.join(ckpt_dir, "latest.tmp"), os.path.join(ckpt_dir, "latest"))
        _prune(ckpt_dir, keep)
    log.info("checkpoint saved: %s", d)
    return d


def _save_flat(d: str, trainer) -> list:
    n = trainer._master.numel()
    pieces = []
    for k, lo in enumerate(range(0, n, PIECE_ELEMS)):
        hi = min(n, lo + PIECE_ELEMS)
        _write(os.path.join(d, "optim", f"part_{k:05d}.safetensors"),
               {"master": trainer._master[lo:hi], "m": trainer.m[lo:hi], "v": trainer.v[lo:hi]})
        pieces.append([lo, hi])
    return pieces


def _save_model(d: str, model) -> list:
    """Trainable weights by name, in files of <= 2 x PIECE_ELEMS elements."""
    parts, cur, size = [], {}, 0

    def flush():
        nonlocal cur, size
        if cur:
            name = f"part_{len(parts):05d}.safetensors"
            _write(os.path.join(d, "model", name), cur)
            parts.append(name)
        cur, size = {}, 0

    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if size and size + p.numel() > 2 * PIECE_ELEMS:
            flush()
        cur[n] = p
        size += p.numel()
    flush()
    return parts


def _save_zero3(d: str, tr, rank: int) -> list:
    table = []
    for u in tr.units:
        off = u.master_view.storage_offset() - tr.master.storage_offset()
        sl = slice(off, off + u.shard_numel)
        _write(os.path.join(d, "z3", f"rank_{rank}", f"unit_{u.uid:04d}.safetensors"),
               {"master": tr.master[sl], "m": tr.m[sl], "v": tr.v[sl]})
        table.append({"uid": u.uid, "names": u.names, "numels": u.numels, "numel": u.numel,
                      "full_numel": u.full_numel, "shard_numel": u.shard_numel,
                      "replicated": bool(getattr(u, "replicated", False))})
    return table


def _prune(ckpt_dir: str, keep: int):
    steps = sorted(int(n.split("_")[1]) for n in os.listdir(ckpt_dir) if n.startswith("step_"))
    for s in steps[:-keep] if keep > 0 else []:
        shutil.rmtree(os.path.join(ckpt_dir, f"step_{s}"), ignore_errors=True)


def latest_step(ckpt_dir: str) -> int | None:
    p = os.path.join(ckpt_dir, "latest")
    if not os.path.exists(p):
        return None
    try:
        return int(open(p).read().strip())
    except ValueError:
        return None


# ---------------------------------------------------------------------- load
def load(ckpt_dir: str, trainer, step: int | None = None) -> dict | None:
    """Restore trainer state; returns the manifest's ``extra`` dict (or None)."""
    step = latest_step(ckpt_dir) if step is None else step
    if step is None:
        return None
    d = os.path.join(ckpt_dir, f"step_{step}")
    with open(os.path.join(d, "manifest.json")) as f:
        man = json.load(f)
    rank, world = _rank_world()
    kind = _kind(trainer)
    if hasattr(trainer, "params_ready"):
        trainer.params_ready()
    if man.get("format", 1) < 2:
        _load_v1(d, man, trainer, rank, world)
    elif man["kind"] != kind:
        raise RuntimeError(f"checkpoint written by a {man['kind']} trainer, resuming with {kind}")
    elif kind == "zero3":
        _load_zero3(d, man, trainer, rank, world)
        trainer.finish_load(man["step"])
    elif kind == "zero1":
        if man["world_size"] != world:
            raise RuntimeError(f"ZeRO-1 checkpoint written with world {man['world_size']}, resuming with {world}")
        _require_same_layout(man.get("layout"), trainer.flat.state_dict(), "ZeRO-1")
        sd = {k: v.to(trainer._master.device) for k, v in load_file(os.path.join(d, f"rank_{rank}.safetensors")).items()}
        sd["step"] = man["step"]
        trainer.load_state_dict(sd)
    else:
        segs = _remap_segments(man["layout"], trainer.flat.state_dict())
        for k, (lo, hi) in enumerate(man["pieces"]):
            with safe_open(os.path.join(d, "optim", f"part_{k:05d}.safetensors"), framework="pt") as f:
                for key, dst in (("master", trainer._master), ("m", trainer.m), ("v", trainer.v)):
                    sl = f.get_slice(key)
                    for olo, ohi, nlo in segs:
                        a, b = max(olo, lo), min(ohi, hi)
                        if a < b:
                            dst[nlo + a - olo:nlo + b - olo].copy_(sl[a - lo:b - lo])
        trainer.finish_load(man["step"])
    log.info("resumed from %s", d)
    return man.get("extra", {})


def _norm_slots(layout: dict | None):
    """Slot table as a list of lists (the manifest's JSON lists and the live tuples compare equal)."""
    return None if not layout else [list(x) for x in layout.get("slots", [])]


def _require_same_layout(old: dict | None, new: dict, what: str) -> None:
    """Sharded optimizer state is a raw copy of flat ranges: it is only valid into the SAME flat
    layout (the round-3 bucket order moved slots, so an older sharded file would have
    landed on the wrong parameters without an error)."""
    if not old:
        raise RuntimeError(f"{what} checkpoint has no layout record; cannot verify the flat layout")
    if _norm_slots(old) != _norm_slots(new) or old.get("numel") != new.get("numel"):
        raise RuntimeError(f"{what} checkpoint was written with a different flat-buffer layout (parameter order / "
                           "bucketing changed); resume it with the trainer version that wrote it, or re-save it "
                           "unsharded (DDP) so it can be remapped by parameter name")


def _remap_segments(old: dict | None, new: dict) -> list:
    """(old_lo, old_hi, new_lo) flat ranges moving every slot, by name, from the
    checkpoint's layout to the current one (identity when they agree)."""
    if not old or _norm_slots(old) == _norm_slots(new):
        return [(0, new["numel"], 0)]
    where = {name: (off, n) for name, off, n, _ in old["slots"]}
    segs = []
    for name, off, n, _ in new["slots"]:
        if name not in where or where[name][1] != n:
            raise RuntimeError(f"checkpoint has no parameter {name} of {n} elements")
        segs.append((where[name][0], where[name][0] + n, off))
    return segs


def _load_v1(d, man, trainer, rank, world):
    """Round-1/2 format: one rank_<r>.safetensors per writer with whole flat buffers."""
    src = rank if man.get("sharded") else 0
    if man.get("sharded") and man.get("world_size") != world:
        raise RuntimeError(f"sharded checkpoint written with world {man['world_size']}, resuming with {world}")
    if man.get("sharded") and hasattr(trainer, "flat"):
        _require_same_layout(man.get("layout"), trainer.flat.state_dict(), "sharded (v1)")
    tensors = load_file(os.path.join(d, f"rank_{src}.safetensors"))
    dev = trainer.flat.master.device if hasattr(trainer, "flat") else trainer.master.device
    if hasattr(trainer, "flat") and not man.get("sharded") and man.get("layout"):
        segs = _remap_segments(man["layout"], trainer.flat.state_dict())
        sd = {}
        for key, like in (("master", trainer._master), ("m", trainer.m), ("v", trainer.v)):
            out = torch.zeros(like.numel(), dtype=torch.float32, device=like.device)
            for olo, ohi, nlo in segs:
                out[nlo:nlo + ohi - olo].copy_(tensors[key][olo:ohi])
            sd[key] = out
    else:
        sd = {k: v.to(dev) for k, v in tensors.items()}
    sd["step"] = man["step"]
    trainer.load_state_dict(sd)


def _load_zero3(d, man, tr, rank, world):
    """Every unit's new shard [r S', (r+1) S') read out of the old ranks' shard
    files: the unit's flat content [0, numel) is world-independent, only the
    padding and the cut points change."""
    old_world = man["world_size"]
    table = {e["uid"]: e for e in man["units"]}
    for u in tr.units:
        e = table.get(u.uid)
        if e is None or e["names"] != u.names or e["numel"] != u.numel:
            raise RuntimeError(f"checkpoint unit {u.uid} does not match the model ({u.names[:2]}...)")
        S_old = e["shard_numel"]
        # a replicated unit (every rank holds all of it) was written whole by every rank: read
        # rank 0's copy; a unit replicated now takes the whole content [0, numel)
        old_q = 1 if e.get("replicated") else old_world
        if e.get("replicated"):
            S_old = e["numel"]
        off = u.master_view.storage_offset() - tr.master.storage_offset()
        r = 0 if getattr(u, "replicated", False) else rank
        a0, a1 = r * u.shard_numel, min((r + 1) * u.shard_numel, u.numel)
        for buf in (tr.master, tr.m, tr.v):
            buf[off:off + u.shard_numel].zero_()
        for q in range(old_q):
            lo, hi = max(a0, q * S_old), min(a1, (q + 1) * S_old)
            if lo >= hi:
                continue
            path = os.path.join(d, "z3", f"rank_{q}", f"unit_{u.uid:04d}.safetensors")
            with safe_open(path, framework="pt") as f:
                for key, buf in (("master", tr.master), ("m", tr.m), ("v", tr.v)):
                    src = f.get_slice(key)[lo - q * S_old:hi - q * S_old]
                    buf[off + lo - a0:off + hi - a0].copy_(src)


def load_model_weights(model, path: str) -> None:
    """Load named weights: our model.safetensors / model/ directory, a step
    directory (format 2: its ``model/`` parts; ZeRO-3: assembled from the unit
    shards of every rank, one unit at a time), or any .safetensors of named weights."""
    named = dict(model.named_parameters())
    files = [path]
    if os.path.isdir(path):
        man_p = os.path.join(path, "manifest.json")
        if os.path.exists(man_p):
            with open(man_p) as f:
                man = json.load(f)
            if man.get("kind") == "zero3":
                _load_zero3_weights(path, man, named)
                _refresh(model)
                return
            if os.path.isdir(os.path.join(path, "model")):
                path = os.path.join(path, "model")
            elif os.path.exists(os.path.join(path, "model.safetensors")):
                path = os.path.join(path, "model.safetensors")
        files = ([os.path.join(path, f) for f in sorted(os.listdir(path)) if f.endswith(".safetensors")]
                 if os.path.isdir(path) else [path])
    with torch.no_grad():
        for fp in files:
            for k, v in load_file(fp).items():
                if k in named:
                    named[k].copy_(v.to(named[k].device, named[k].dtype))
    _refresh(model)


def _load_zero3_weights(d: str, man: dict, named: dict):
    world = man["world_size"]
    with torch.no_grad():
        for e in man["units"]:
            S = e["shard_numel"]
            full = torch.cat([load_file(os.path.join(d, "z3", f"rank_{q}", f"unit_{e['uid']:04d}.safetensors"))
                              ["master"][:S] for q in range(1 if e.get("replicated") else world)])
            o = 0
            for name, n in zip(e["names"], e["numels"]):
                if name in named:
                    p = named[name]
                    p.copy_(full[o:o + n].view(p.shape).to(p.device, p.dtype))
                o += n
            del full


def _refresh(model):
    if hasattr(model, "sync_adapters_"):
        model.sync_adapters_()
    if hasattr(model, "refresh_images_"):
        model.refresh_images_()
