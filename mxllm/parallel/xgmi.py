"""Intra-node peer-memory collectives for tiny messages.

The reference's only collective is a 1-element NCCL barrier
(reference src/distributed_inference.py:18).  In mxllm the latency-bound
collectives — the loss / token-count / grad-norm scalars logged each step,
the parameter-checksum desync check (A6/C8) and device-side barriers — go
through :class:`XgmiComm`: a HIP one-shot kernel (``csrc/kernels/xgmi.hip``)
that writes each rank's values straight into every peer's uncached buffer
over the xGMI mesh and reduces locally after a system-scope flag.  Buffers
are exchanged once with ``hipIpcGetMemHandle``/``hipIpcOpenMemHandle`` through
the process group.  RCCL remains the path for bulk traffic (DDP buckets,
ZeRO-3 gathers) and for anything that crosses nodes.

OPT-IN (``MXLLM_XGMI=1``): peer mapping across two DISTINCT GPUs has only been
exercised as two processes on one GPU (the test boxes have one GPU), so by
default :func:`create` returns ``None`` and callers use RCCL.  When enabled it
is used only when every rank of the group lives on this host
(``LOCAL_WORLD_SIZE == WORLD_SIZE``) and all ranks use GPUs, and it is
all-or-none across the ranks (any local failure: every rank falls back).
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("mxllm.xgmi")

_OPS = {"sum": 0, "max": 1, "min": 2}


class XgmiComm:
    def __init__(self, rank: int, world: int, device: torch.device, *, max_elems: int = 16384,
                 timeout_s: float | None = None):
        """Local half only (allocate + export the IPC handle); :func:`create`
        exchanges handles and calls :meth:`open` on every rank."""
        from ..ops._ext import native

        native()
        if timeout_s is None:
            timeout_s = float(os.environ.get("MXLLM_XGMI_TIMEOUT_S", "300"))
        self.rank, self.world, self.device, self.timeout_s = rank, world, device, float(timeout_s)
        self._c = torch.classes.mxllm.XgmiComm(rank, world, device.index, max_elems, float(timeout_s))
        self.max_elems = max_elems

    def handle(self) -> list[int]:
        return self._c.handle().tolist()

    def open(self, handles: list[list[int]]):
        self._c.open(torch.tensor(handles, dtype=torch.uint8))

    def self_test(self, timeout_s: float = 20.0) -> bool:
        """One short-timeout all-reduce of known values on every rank; a peer
        whose writes are not visible shows up here instead of mid-training."""
        self._c.set_timeout(timeout_s)
        try:
            t = torch.arange(4, dtype=torch.float32, device=self.device) + self.rank
            self.all_reduce_(t, "sum")
            m = torch.full((1,), float(self.rank), device=self.device)
            self.all_reduce_(m, "max")
            got = t.tolist() + m.tolist()
            base = self.world * (self.world - 1) / 2
            want = [base + i * self.world for i in range(4)] + [float(self.world - 1)]
            ok = got == want and not self._c.error()
            if not ok:
                log.warning("xGMI self-test mismatch on rank %d: %s != %s", self.rank, got, want)
            return ok
        finally:
            self._c.clear_error()
            self._c.set_timeout(self.timeout_s)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce of a small float32 tensor on this rank's GPU
        (enqueued on the current stream; no host sync)."""
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("XgmiComm.all_reduce_ expects a contiguous float32 tensor")
        self._c.all_reduce_(t, _OPS[op])
        return t

    def barrier(self, sync: bool = True):
        self._c.barrier()
        if sync:
            torch.cuda.current_stream(self.device).synchronize()
            self.check()

    def check(self):
        if self._c.error():
            raise RuntimeError("xGMI collective timed out waiting for a peer (MXLLM_XGMI_TIMEOUT_S)")

    def close(self):
        self._c.close()


class XgmiGraphComm:
    """Graph-safe bf16 sum all-reduce over peer memory (tensor-parallel decode):
    device-resident epochs, so the launch can be captured into a hipGraph and
    replayed.  ``csrc/kernels/xgmi.hip`` ``mx_xgmi_allreduce_bf16``."""

    def __init__(self, rank: int, world: int, device: torch.device, *, max_elems: int = 1 << 19,
                 timeout_s: float | None = None):
        from ..ops._ext import native

        native()
        if timeout_s is None:
            timeout_s = float(os.environ.get("MXLLM_XGMI_TIMEOUT_S", "300"))
        self.rank, self.world, self.device, self.timeout_s = rank, world, device, float(timeout_s)
        self.max_elems = max_elems
        self._c = torch.classes.mxllm.XgmiGraphComm(rank, world, device.index, max_elems, float(timeout_s))

    def handle(self) -> list[int]:
        return self._c.handle().tolist()

    def open(self, handles: list[list[int]]):
        self._c.open(torch.tensor(handles, dtype=torch.uint8))

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype == torch.bfloat16 and t.is_contiguous() and t.device == self.device
                and 0 < t.numel() <= self.max_elems and t.numel() % 8 == 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        self._c.all_reduce_(t)
        return t

    def self_test(self, timeout_s: float = 20.0) -> bool:
        self._c.set_timeout(timeout_s)
        try:
            n = 4096 + 8
            t = (torch.arange(n, device=self.device) % 7 + self.rank).to(torch.bfloat16)
            self.all_reduce_(t)
            want = ((torch.arange(n, device=self.device) % 7) * self.world
                    + self.world * (self.world - 1) / 2).to(torch.bfloat16)
            ok = bool(torch.equal(t, want)) and not self._c.error()
            if not ok:
                log.warning("xGMI bf16 self-test mismatch on rank %d", self.rank)
            return ok
        finally:
            self._c.clear_error()
            self._c.set_timeout(self.timeout_s)

    def check(self):
        if self._c.error():
            raise RuntimeError("xGMI bf16 all-reduce timed out waiting for a peer (MXLLM_XGMI_TIMEOUT_S)")

    def close(self):
        self._c.close()


def eligible(group=None) -> bool:
    if os.environ.get("MXLLM_XGMI", "0") != "1" or not dist.is_initialized():
        return False
    if not torch.cuda.is_available() or os.environ.get("MXLLM_FORCE_CPU") == "1":
        return False
    world = dist.get_world_size(group)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return 1 < world <= 16 and local_world == world


def create(device: torch.device, group=None, cls=XgmiComm, **kw):
    """Collective over ``group``: every rank must call it.  Returns a
    communicator (``cls``: XgmiComm or XgmiGraphComm) on every rank, or
    ``None`` on every rank (never a mix, so all ranks keep issuing the same
    collectives) when peer memory is not usable."""
    if not eligible(group):
        return None
    world = dist.get_world_size(group)
    comm, handle = None, None
    try:
        comm = cls(dist.get_rank(group), world, device, **kw)
        handle = comm.handle()
    except Exception as e:  # noqa: BLE001
        log.warning("xGMI communicator: local setup failed (%s)", e)
    handles: list = [None] * world
    dist.all_gather_object(handles, handle, group=group)
    ok = all(h is not None for h in handles)
    if ok:
        try:
            comm.open(handles)
            ok = comm.self_test()
        except Exception as e:  # noqa: BLE001  (e.g. IPC not permitted)
            log.warning("xGMI communicator: opening peer buffers failed (%s)", e)
            ok = False
    oks: list = [None] * world
    dist.all_gather_object(oks, ok, group=group)
    if not all(oks):
        if comm is not None:
            comm.close()
        log.warning("xGMI peer-memory communicator unavailable; small collectives use RCCL")
        return None
    return comm
