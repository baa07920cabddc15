"""Flat parameter/gradient storage.

Every trainable parameter becomes a view into ONE contiguous buffer (and its
gradient a view into one contiguous grad buffer) laid out in *reverse
registration order* — the order autograd produces gradients — so DDP buckets
are plain contiguous slices that fill front to back during backward, the
fused AdamW is one kernel over the whole buffer, and checkpoints are a single
tensor per state.  Slices are padded to 64 elements (256 B of f32) so every
bucket boundary is aligned for 16-B vector access.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 64


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class Slot:
    name: str
    offset: int
    numel: int
    shape: tuple


class FlatParams:
    """Owns param (compute dtype), optional fp32 master, and grad buffers.

    ``param_dtype``: storage of the live parameters the model computes with.
    ``master``: fp32 copy (created when param_dtype != fp32).
    ``grad_dtype``: dtype of the flat grad buffer (defaults to param dtype);
    float32 with bf16 parameters = fp32 gradient accumulation and reduction.
    ``split_master``: the fp32 master is a :class:`mxllm.ops.SplitMaster` over
    ``params`` (exact fp32 values, 2 B/param less state and optimizer traffic).
    """

    def __init__(self, named_params: list[tuple[str, torch.nn.Parameter]], grad_dtype: torch.dtype | None = None,
                 reverse: bool = True, align: int = ALIGN, split_master: bool = False):
        if not named_params:
            raise ValueError("no trainable parameters")
        order = list(reversed(named_params)) if reverse else list(named_params)
        dev = order[0][1].device
        pdt = order[0][1].dtype
        if any(p.dtype != pdt for _, p in order):
            raise ValueError("all trainable parameters must share one dtype")
        self.slots: list[Slot] = []
        off = 0
        for n, p in order:
            self.slots.append(Slot(n, off, p.numel(), tuple(p.shape)))
            off += _round(p.numel(), align)
        self.numel = off
        self.device = dev
        self.param_dtype = pdt
        self.params = torch.zeros(off, dtype=pdt, device=dev)
        self.grad_dtype = grad_dtype or pdt
        self.grads = torch.zeros(off, dtype=self.grad_dtype, device=dev)
        self._plist = []
        with torch.no_grad():
            for (n, p), s in zip(order, self.slots):
                view = self.params[s.offset:s.offset + s.numel].view(s.shape)
                view.copy_(p.data)
                p.data = view
                self._plist.append(p)
        if pdt == torch.float32:
            self.master = self.params
        elif split_master:  # fp32 master = (params, int16 low halves): no separate bf16 copy
            from ..ops.optim import SplitMaster

            self.master = SplitMaster(self.params)
        else:
            self.master = self.params.float()
        # fp32 gradients of low-precision parameters (autograd cannot hold them in
        # ``.grad``): ops add into ``p._mx_grad32`` (grad_ready.accum_grad / the
        # fp32-output dW GEMMs), anything autograd accumulates in ``.grad`` is folded
        # in by a hook that runs before every other post-accumulate hook (DDP's)
        self.grad32 = self.grad_dtype == torch.float32 and pdt != torch.float32
        if self.grad32:
            for p in self._plist:
                p.register_post_accumulate_grad_hook(self._fold_hook)
        self.attach_grads()

    def _view(self, k: int, buf: torch.Tensor) -> torch.Tensor:
        s = self.slots[k]
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def _fold_hook(self, p):
        if p.grad is not None:
            if getattr(p, "_mx_grad_fresh", False):
                p._mx_grad32.copy_(p.grad)
                p._mx_grad_fresh = False
            else:
                p._mx_grad32.add_(p.grad)
            p.grad = None

    def zero_unwritten_(self):
        """Zero the slots of parameters still flagged ``_mx_grad_fresh`` after a
        backward (no op wrote their gradient: unused this step)."""
        for k, p in enumerate(self._plist):
            if getattr(p, "_mx_grad_fresh", False):
                self._view(k, self.grads).zero_()
                p._mx_grad_fresh = False

    def attach_grads(self):
        """Point every ``p.grad`` (fp32 mode: ``p._mx_grad32``) at its slice of
        the flat grad buffer."""
        for k, p in enumerate(self._plist):
            g = self._view(k, self.grads)
            if self.grad32:
                p._mx_grad32 = g
                continue
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g if self.grad_dtype == p.dtype else None
        return self

    @property
    def param_list(self):
        return self._plist

    def zero_grad(self):
        self.grads.zero_()
        self.attach_grads()

    def sync_grads_from_params(self) -> list[int]:
        """If autograd replaced a .grad (dtype mismatch / detached), copy it back
        (fp32 mode: fold any ``.grad`` left behind into the fp32 buffer).  Returns
        the indices of the slots written here."""
        changed = []
        for k, (p, s) in enumerate(zip(self._plist, self.slots)):
            g = p.grad
            if g is None:
                continue
            if self.grad32:
                self._fold_hook(p)
                changed.append(k)
                continue
            flat = self.grads[s.offset:s.offset + s.numel]
            if g.data_ptr() != flat.data_ptr():
                flat.copy_(g.reshape(-1))
                p.grad = flat.view(s.shape)
                changed.append(k)
        return changed

    def state_dict(self):
        return {"slots": [(s.name, s.offset, s.numel, list(s.shape)) for s in self.slots], "numel": self.numel}


def production_order(model, named: list) -> list:
    """Trainable parameters in gradient-PRODUCTION order (the flat-buffer layout):
    the model's forward parameter groups (``Llama._wait_groups``: embedding, each
    layer + the norm it applies next, head) reversed, each group reversed — the LM
    head's gradient comes first in backward, the embedding's last.  DDP buckets then
    fill front to back during backward (the head's 1 GB bucket no longer waits for
    the embedding), and every forward group is one contiguous range (the
    per-layer optimizer chunks).  Parameters outside the groups keep registration
    order (reversed) at the end."""
    groups_fn = getattr(model, "_wait_groups", None)
    if groups_fn is None:
        return list(reversed(named))
    want = {id(p): (n, p) for n, p in named}
    taken, chunks = set(), []
    for g in groups_fn():
        c = [want[id(p)] for p in g if id(p) in want and id(p) not in taken]
        taken.update(id(p) for _, p in c)
        chunks.append(c)
    out = [e for c in reversed(chunks) for e in reversed(c)]
    out += [e for e in reversed(named) if id(e[1]) not in taken]
    return out
