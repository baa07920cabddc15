"""Checkpoint / resume — safetensors + JSON manifest.

Layout ``<dir>/step_<N>/``:
  manifest.json                step, world layout, parallel mode, flat-buffer
                               slot table, data-loader state, RNG seeds
  rank_<r>.safetensors         optimizer state (master/m/v flat buffers) of rank r
                               (DDP: rank 0 only — replicas are identical;
                               ZeRO-3: every rank's own shard)
  model.safetensors            trainable weights by name (LoRA adapters, or the
                               full model for full fine-tuning) — loadable by
                               ``load_model_weights`` for serving
``<dir>/latest`` holds the newest complete step (written last = atomic commit).
Only safetensors/JSON are used: nothing is ever unpickled.
"""
from __future__ import annotations

import json
import logging
import os
import shutil

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file

log = logging.getLogger("mxllm.ckpt")


def _rank_world():
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def save(ckpt_dir: str, trainer, step: int, extra: dict | None = None, sharded: bool = False, keep: int = 2) -> str:
    rank, world = _rank_world()
    d = os.path.join(ckpt_dir, f"step_{step}")
    if rank == 0:
        os.makedirs(d, exist_ok=True)
    if dist.is_initialized():
        dist.barrier()
    sd = trainer.state_dict()
    if sharded or rank == 0:
        tensors = {k: v.detach().contiguous().cpu() for k, v in sd.items() if isinstance(v, torch.Tensor)}
        save_file(tensors, os.path.join(d, f"rank_{rank}.safetensors"))
    if rank == 0:
        weights = {n: p.detach().contiguous().cpu() for n, p in trainer.model.named_parameters() if p.requires_grad}
        if weights and not sharded:
            save_file(weights, os.path.join(d, "model.safetensors"))
        man = {"step": step, "world_size": world, "sharded": sharded,
               "layout": sd.get("layout"), "extra": extra or {}}
        with open(os.path.join(d, "manifest.json"), "w") as f:
            json.dump(man, f, indent=1)
    if dist.is_initialized():
        dist.barrier()
    if rank == 0:
        with open(os.path.join(ckpt_dir, "latest.tmp"), "w") as f:
            f.write(str(step))
        os.replace(os.path.join(ckpt_dir, "latest.tmp"), os.path.join(ckpt_dir, "latest"))
        _prune(ckpt_dir, keep)
    log.info("checkpoint saved: %s", d)
    return d


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


def load(ckpt_dir: str, trainer, step: int | None = None) -> dict | None:
    """Restore trainer state; returns the manifest's ``extra`` dict (or None)."""
    step = latest_step(ckpt_dir) if step is None else step
    if step is None:
        return None
    d = os.path.join(ckpt_dir, f"step_{step}")
    with open(os.path.join(d, "manifest.json")) as f:
        man = json.load(f)
    rank, world = _rank_world()
    src = rank if man.get("sharded") else 0
    if man.get("sharded") and man.get("world_size") != world:
        raise RuntimeError(f"sharded checkpoint written with world {man['world_size']}, resuming with {world}")
    tensors = load_file(os.path.join(d, f"rank_{src}.safetensors"))
    dev = trainer.flat.master.device if hasattr(trainer, "flat") else trainer.master.device
    sd = {k: v.to(dev) for k, v in tensors.items()}
    sd["step"] = man["step"]
    trainer.load_state_dict(sd)
    log.info("resumed from %s", d)
    return man.get("extra", {})


def load_model_weights(model, path: str) -> None:
    """Load named weights (our model.safetensors, or a directory of them)."""
    files = [path]
    if os.path.isdir(path):
        files = [os.path.join(path, f) for f in sorted(os.listdir(path)) if f.endswith(".safetensors")]
    named = dict(model.named_parameters())
    with torch.no_grad():
        for fp in files:
            for k, v in load_file(fp).items():
                if k in named:
                    named[k].copy_(v.to(named[k].device, named[k].dtype))
        if hasattr(model, "sync_adapters_"):
            model.sync_adapters_()
        if hasattr(model, "refresh_images_"):
            model.refresh_images_()
