"""Cross-rank desynchronisation detector.

The reference's troubleshooting guide tells users to keep seeds consistent
across nodes (reference docs/troubleshooting.md:57-62) but nothing checks it.
mxllm initialises every rank from the same seed instead of broadcasting 16 GB
of weights, so it must be able to prove the replicas agree:

``param_checksum`` reduces a tensor's raw bits to an exact integer (the
buffer viewed as int16 words, summed in int64 with position weights, so any
flipped bit or permuted value changes it and the sum is order independent);
``check_in_sync`` all-reduces that checksum with MAX and MIN (xGMI one-shot
kernel on a GPU node, gloo/RCCL otherwise) and reports ranks that disagree.
"""
from __future__ import annotations

import logging

import torch
import torch.distributed as dist

from . import runtime

log = logging.getLogger("mxllm.consistency")

_CHUNK_BITS = 20  # f32 holds integers < 2^24 exactly; pieces of 20 bits stay exact


def param_checksum(t: torch.Tensor, chunk: int = 1 << 26) -> int:
    """Exact, order-independent integer fingerprint of ``t``'s bits (streamed
    in chunks so an 8B-element buffer needs no 64 GB int64 copy)."""
    flat = t.detach().contiguous().view(-1)
    words = flat.view(torch.int16) if flat.element_size() % 2 == 0 else flat.view(torch.uint8).to(torch.int16)
    total = torch.zeros((), dtype=torch.int64, device=words.device)
    for s in range(0, words.numel(), chunk):
        w = words[s:s + chunk].to(torch.int64)
        idx = torch.arange(s, s + w.numel(), device=w.device, dtype=torch.int64)
        total += ((w + 40503) * ((idx % 65521) + 1)).sum()  # position-weighted: swaps change it
    return int(total.item()) & ((1 << 60) - 1)


def _pieces(v: int) -> list[float]:
    return [float((v >> (_CHUNK_BITS * i)) & ((1 << _CHUNK_BITS) - 1)) for i in range(3)]


def check_in_sync(tensors, *, raise_on_mismatch: bool = True, what: str = "parameters") -> bool:
    """True when every rank holds bit-identical ``tensors`` (a tensor or a list)."""
    if isinstance(tensors, torch.Tensor):
        tensors = [tensors]
    cs = 0
    for t in tensors:
        cs = (cs * 1000003 + param_checksum(t)) & ((1 << 60) - 1)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return True
    mine = _pieces(cs)
    hi = runtime.all_reduce_scalars(mine, op="max")
    lo = runtime.all_reduce_scalars(mine, op="min")
    ok = hi == lo
    if not ok:
        msg = (f"rank {dist.get_rank()}: {what} differ across ranks (checksum pieces mine={mine} "
               f"max={hi} min={lo}); check seeds / deterministic init / skipped all-reduce")
        log.error(msg)
        if raise_on_mismatch:
            raise RuntimeError(msg)
    return ok
