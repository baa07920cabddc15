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
    ``grad_dtype``: dtype of the flat grad buffer (defaults to param dtype).
    """

    def __init__(self, named_params: list[tuple[str, torch.nn.Parameter]], grad_dtype: torch.dtype | None = None,
                 reverse: bool = True, align: int = ALIGN):
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
        self.master = self.params if pdt == torch.float32 else self.params.float()
        self.attach_grads()

    def attach_grads(self):
        """Point every ``p.grad`` at its slice of the flat grad buffer."""
        for p, s in zip(self._plist, self.slots):
            g = self.grads[s.offset:s.offset + s.numel].view(s.shape)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g if self.grad_dtype == p.dtype else None
        return self

    @property
    def param_list(self):
        return self._plist

    def zero_grad(self):
        self.grads.zero_()
        self.attach_grads()

    def sync_grads_from_params(self):
        """If autograd replaced a .grad (dtype mismatch / detached), copy it back."""
        for p, s in zip(self._plist, self.slots):
            g = p.grad
            if g is None:
                continue
            flat = self.grads[s.offset:s.offset + s.numel]
            if g.data_ptr() != flat.data_ptr():
                flat.copy_(g.reshape(-1))
                p.grad = flat.view(s.shape)

    def state_dict(self):
        return {"slots": [(s.name, s.offset, s.numel, list(s.shape)) for s in self.slots], "numel": self.numel}
