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
                 bucket_mb: float = 128.0, first_bucket_mb: float = 16.0, broadcast_init: bool = False):
        self.model = model
        self.env = env
        self.opt = optim or OptimConfig()
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.flat = FlatParams(named)
        self.ddp = DDP(self.flat, bucket_mb=bucket_mb, first_bucket_mb=first_bucket_mb)
        if broadcast_init:
            self.ddp.broadcast_params(0)
        self._sync_adapters()
        self.m = torch.zeros_like(self.flat.master)
        self.v = torch.zeros_like(self.flat.master)
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
        if o.grad_clip and o.grad_clip > 0:
            # global grad norm on device; the clip coefficient is applied inside
            # the fused AdamW kernel via grad_scale (host read only for logging)
            sq = ops.sq_norm(self.flat.grads)
            gnorm = sq.sqrt() * scale
            self.last_grad_norm = gnorm
            coef = torch.clamp(o.grad_clip / (gnorm + 1e-6), max=1.0)
            gscale = coef * scale
        else:
            gscale = scale
        ops.adamw_step_(self.flat.master, self.flat.grads, self.m, self.v, self.lowp, lr=o.lr_at(self.step_num),
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
    def state_dict(self) -> dict:
        return {"step": self.step_num, "master": self.flat.master, "m": self.m, "v": self.v,
                "layout": self.flat.state_dict()}

    def load_state_dict(self, sd: dict):
        self.step_num = int(sd["step"])
        self.flat.master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.flat.master is not self.flat.params:
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
