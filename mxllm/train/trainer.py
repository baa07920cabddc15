"""Training step: forward -> fused CE -> backward (bucketed RCCL all-reduce
overlapped via DDP hooks) -> grad-norm clip -> fused AdamW over flat buffers.

This is the real version of the reference's simulated ``process_batch``
(reference src/utils.py:12-23): the loss is computed from the
model's own logits and gradients flow into an optimizer step.
"""
from __future__ import annotations

import logging
import math
import time
from dataclasses import dataclass

import torch

from .. import ops
from ..parallel.ddp import DDP
from ..parallel.flat import FlatParams
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


class Trainer:
    def __init__(self, model: torch.nn.Module, env: DistEnv, optim: OptimConfig | None = None, *,
                 bucket_mb: float = 128.0, first_bucket_mb: float = 16.0, broadcast_init: bool = False,
                 shard_optimizer: bool = False):
        """``shard_optimizer``: ZeRO-1 (mxllm/parallel/zero1.py) — gradients are
        reduce-scattered, each rank updates its 1/N slice, parameters are
        all-gathered back.  At world 1 it is plain DDP (nothing to shard)."""
        self.model = model
        self.env = env
        self.opt = optim or OptimConfig()
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        world = env.world_size
        self.zero1 = None
        if shard_optimizer and world > 1:
            from ..parallel.zero1 import Zero1

            self.flat = FlatParams(named, align=64 * world)
            self.ddp = self.zero1 = Zero1(self.flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb)
            self._master = self.zero1.master
            if getattr(model, "param_wait", "absent") is None:
                model.param_wait = self.zero1.wait_params  # per-layer wait in the next forward
        else:
            self.flat = FlatParams(named)
            self.ddp = DDP(self.flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb)
            self._master = self.flat.master
        if broadcast_init:
            self.ddp.broadcast_params(0)
        self._sync_adapters()
        self.m = torch.zeros_like(self._master)
        self.v = torch.zeros_like(self._master)
        self.step_num = 0
        self.last_grad_norm: torch.Tensor | None = None

    @property
    def lowp(self):
        return None if self.flat.master is self.flat.params else self.flat.params

    def train_step(self, micro_batches: list[tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """One optimizer step over ``micro_batches`` [(ids, labels), ...].
        Returns the mean loss as a device tensor (no host sync)."""
        n = len(micro_batches)
        self.model.train()
        if self.zero1 is not None and getattr(self.model, "param_wait", None) is None:
            self.zero1.wait_params()  # model without per-layer waits: all parameters first
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
        self.flat.sync_grads_from_params()
        with range_("grad_allreduce_wait"):
            scale = self.ddp.finish() / n if n > 1 else self.ddp.finish()
        self.step_num += 1
        with range_("optimizer"):
            self._optimizer_step(scale)
        return total / n

    def _optimizer_step(self, scale: float):
        o = self.opt
        z = self.zero1
        grads = z.gshard if z is not None else self.flat.grads
        if o.grad_clip and o.grad_clip > 0:
            # global grad norm on device; the clip coefficient is applied inside
            # the fused AdamW kernel via grad_scale (host read only for logging)
            sq = ops.sq_norm(grads)
            if z is not None:
                from ..parallel.runtime import all_reduce_small_

                all_reduce_small_(sq)  # sum of the shards' squares
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
        else:
            ops.adamw_step_(self.flat.master, grads, self.m, self.v, self.lowp, lr=o.lr_at(self.step_num),
                            beta1=o.beta1, beta2=o.beta2, eps=o.eps, weight_decay=o.weight_decay,
                            step=self.step_num, grad_scale=gscale, zero_grad=True)  # grads cleared in the same pass
        self._sync_adapters()
        self.flat.attach_grads()

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
        return {"step": self.step_num, "master": self._master, "m": self.m, "v": self.v,
                "layout": self.flat.state_dict()}

    def load_state_dict(self, sd: dict):
        self.step_num = int(sd["step"])
        self._master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        z = self.zero1
        if z is not None:
            if z.master is not z.pshard:
                z.pshard.copy_(z.master)
            z.gather_params()
            z.wait_params()
        elif self.flat.master is not self.flat.params:
            self.flat.params.copy_(self.flat.master)
        self._sync_adapters()


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
