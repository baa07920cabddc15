"""One collective interface for the trainers: RCCL / gloo, or peer memory.

The reference's only collective is a barrier (reference
src/distributed_inference.py:18); the DDP gradient sync it advertises
(reference README.md:7) is mxllm's own (ddp.py, zero1.py, zero3.py).  Every
bulk collective those trainers issue goes through a communicator created
here, with ONE contract — the one ProcessGroupNCCL (= RCCL on ROCm) has:

  * the collective runs on the communicator's own stream, ordered after
    everything already queued on the caller's current stream;
  * ``async_op=True`` returns a work whose ``wait()`` makes the caller's
    CURRENT stream wait for the collective (no host block);
  * every tensor handed to a collective is kept alive (``record_stream``)
    until the collective has finished with it, whatever the caller drops.

Implementations:

  * :class:`TorchCollectives` — ``torch.distributed`` on a process group:
    RCCL over xGMI on GPUs (the default), gloo on CPU.
  * :class:`PeerCollectives` — direct one-hop reduce-scatter / all-gather over
    IPC-mapped peer memory (``csrc/kernels/peer_coll.hip``): every rank pushes
    to all of its peers at once (7 xGMI links on an 8x MI355X node).
    Opt-in with ``MXLLM_COMM=peer``.  Because a "peer" may be the SAME GPU
    mapped by another process, W ranks can share one GPU: that is how the
    multi-rank trainers run with stream-ordered collectives on a 1-GPU box
    (tests/test_multirank_gpu.py), where RCCL refuses two ranks per device.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("mxllm.comm")


def kind_requested() -> str:
    """``MXLLM_COMM``: ``torch`` (default: RCCL / gloo) or ``peer``."""
    return os.environ.get("MXLLM_COMM", "torch").strip().lower() or "torch"


class TorchCollectives:
    """``torch.distributed`` on ``group`` (RCCL on GPUs, gloo on CPU)."""

    def __init__(self, group=None):
        self.pg = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.kind = dist.get_backend(group) if dist.is_initialized() else "none"

    def all_reduce(self, t: torch.Tensor, async_op: bool = False):
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        return dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.pg, async_op=async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        return dist.all_gather_into_tensor(out, inp, group=self.pg, async_op=async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        dist.broadcast(t, src=src, group=self.pg)

    def close(self):
        pass


class PeerWork:
    """RCCL-style work: ``wait()`` orders the caller's current stream after the collective."""

    __slots__ = ("event", "comm")

    def __init__(self, event, comm):
        self.event, self.comm = event, comm

    def wait(self):
        torch.cuda.current_stream(self.comm.device).wait_event(self.event)
        self.comm.check()
        return True

    def is_completed(self) -> bool:
        return self.event.query()


class PeerCollectives:
    """Bulk sum reduce-scatter / all-gather / all-reduce over IPC-mapped peer
    memory (``torch.classes.mxllm.PeerComm``).  Create with :func:`create`
    (collective over ``group``, which also carries the bootstrap exchange).

    fp32 / bf16; sums in fp32 in rank order, so every rank gets identical bits.

    Two schedules (``MXLLM_PEER_ALGO``):

      * ``resident``: ONE kernel per call whose ``wgs`` workgroups each move ``slot_kb`` per peer
        per exchange and spin on the peers' flags between exchanges (they hold their CUs for the
        whole call: profiles/r5j);
      * ``light``: per segment of <= ``MXLLM_PEER_LIGHT_MB`` per peer, a push kernel and a consume
        kernel that exit, with ONE wave waiting on the peers' flags in between
        (csrc/kernels/peer_coll.hip, "CU-light schedule") -- the CUs stay with the compute stream
        while a peer is late.  It also carries fp32 reduce-scatters as bf16 on the wire
        (``reduce_scatter(..., wire=torch.bfloat16)``: half the link bytes; the fp32 rank-ordered
        sum of the bf16-rounded inputs, identical on every rank)."""

    def __init__(self, group, device: torch.device, *, wgs: int | None = None, slot_kb: int | None = None,
                 timeout_s: float | None = None, algo: str | None = None):
        from ..ops._ext import native

        native()
        self.pg = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device
        self.kind = "peer"
        self.wgs = int(wgs or os.environ.get("MXLLM_PEER_WGS", "32"))
        self.slot_bytes = int(slot_kb or os.environ.get("MXLLM_PEER_SLOT_KB", "64")) * 1024
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("MXLLM_PEER_TIMEOUT_S", "300"))
        self.algo = (algo or os.environ.get("MXLLM_PEER_ALGO", "light")).strip().lower()
        if self.algo not in ("light", "resident"):
            raise ValueError(f"MXLLM_PEER_ALGO must be light or resident, not {self.algo!r}")
        light_cap = 0
        if self.algo == "light":  # bytes per (half, source) slot, 4 KB multiple
            light_cap = max(1, int(float(os.environ.get("MXLLM_PEER_LIGHT_MB", "64")) * 2 ** 20) // 4096) * 4096
        self.light_wgs = int(os.environ.get("MXLLM_PEER_LIGHT_WGS", "128"))
        self._c = torch.classes.mxllm.PeerComm(self.rank, self.world, device.index, self.wgs, self.slot_bytes,
                                               self.timeout_s, light_cap, self.light_wgs)
        self.stream = torch.cuda.Stream(device)
        self._broken = False
        self._last = None  # event of the last collective issued (sync_check)

    # ------------------------------------------------------------------ bootstrap
    def handle(self) -> list[int]:
        return self._c.handle().tolist()

    def open(self, handles: list[list[int]]):
        self._c.open(torch.tensor(handles, dtype=torch.uint8))

    def self_test(self, timeout_s: float = 30.0) -> bool:
        """Reduce-scatter + all-gather + all-reduce of known values (both dtypes, a size
        that needs zero padding) with a short timeout: a peer whose writes are not visible
        shows up here, not mid-training."""
        self._c.set_timeout(timeout_s)
        try:
            W, dev = self.world, self.device
            ok = True
            for dt in (torch.float32, torch.bfloat16):
                n = 8 * W * 3
                x = (torch.arange(n, device=dev) % 13 + self.rank).to(dt)
                out = torch.empty(n // W, dtype=dt, device=dev)
                self.reduce_scatter(out, x)
                want = ((torch.arange(n, device=dev) % 13) * W + W * (W - 1) // 2).to(dt).view(W, -1)[self.rank]
                g = torch.empty(n, dtype=dt, device=dev)
                self.all_gather(g, out)
                y = (torch.arange(40, device=dev) % 5 + self.rank).to(dt)
                self.all_reduce(y)
                ywant = ((torch.arange(40, device=dev) % 5) * W + W * (W - 1) // 2).to(dt)
                torch.cuda.current_stream(dev).synchronize()
                ok &= bool(torch.equal(out, want)) and bool(torch.equal(g.view(W, -1)[self.rank], want))
                ok &= bool(torch.equal(y, ywant))
            if self.algo == "light":  # fp32 through a bf16 wire (small integers: exact in bf16)
                n = 8 * W * 3
                x = (torch.arange(n, device=dev) % 13 + self.rank).float()
                out = torch.empty(n // W, device=dev)
                self.reduce_scatter(out, x, wire=torch.bfloat16)
                want = ((torch.arange(n, device=dev) % 13) * W + W * (W - 1) // 2).float().view(W, -1)[self.rank]
                torch.cuda.current_stream(dev).synchronize()
                ok &= bool(torch.equal(out, want))
            ok = ok and not self._c.error()
            if not ok:
                log.warning("peer-memory self-test mismatch on rank %d", self.rank)
            return ok
        finally:
            self._c.clear_error()
            self._c.set_timeout(self.timeout_s)

    # ------------------------------------------------------------------ collectives
    def _vec(self, dtype) -> int:
        """Element granularity of the sizes a call takes (smaller tensors are padded)."""
        return 8 if self.algo == "light" else 16 // torch.empty(0, dtype=dtype).element_size()

    def _issue(self, fn, tensors, async_op: bool):
        if self._broken:
            raise RuntimeError("peer-memory communicator is broken (an earlier collective timed out)")
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._last = ev
        for t in tensors:
            t.record_stream(self.stream)  # the allocator keeps it until the comm stream is past it
        w = PeerWork(ev, self)
        if async_op:
            return w
        w.wait()
        return None

    @staticmethod
    def _fits(t: torch.Tensor, v: int) -> bool:
        return t.is_contiguous() and t.numel() % v == 0 and t.data_ptr() % 16 == 0

    def _rs(self, out: torch.Tensor, inp: torch.Tensor, wire_bf16: bool = False):
        if self.algo == "light":
            self._c.reduce_scatter_light_(out, inp, wire_bf16)
        else:
            self._c.reduce_scatter_(out, inp)

    def _ag(self, out: torch.Tensor, inp: torch.Tensor):
        if self.algo == "light":
            self._c.all_gather_light_(out, inp)
        else:
            self._c.all_gather_(out, inp)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False,
                       wire: torch.dtype | None = None):
        """``wire=torch.bfloat16`` (fp32 tensors, light schedule): bf16 on the wire, fp32 sum of the
        bf16-rounded inputs in rank order (half the bytes of an fp32 reduce-scatter)."""
        W = self.world
        if inp.numel() != W * out.numel() or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: input must hold world x output elements of one dtype")
        wire_bf16 = wire is not None and wire != inp.dtype
        if wire_bf16 and (wire != torch.bfloat16 or inp.dtype != torch.float32 or self.algo != "light"):
            raise ValueError("reduce_scatter: a bf16 wire takes fp32 tensors on the light schedule")
        v = self._vec(inp.dtype)

        def run():
            if self._fits(inp, v) and self._fits(out, v):
                self._rs(out, inp, wire_bf16)
                return
            m = out.numel()
            mp = -(-m // v) * v  # padded chunk: every rank's chunk starts on a 16-B boundary
            ip = torch.zeros(W, mp, dtype=inp.dtype, device=self.device)
            ip[:, :m].copy_(inp.view(W, m))
            op = torch.empty(mp, dtype=out.dtype, device=self.device)
            self._rs(op, ip.view(-1), wire_bf16)
            out.copy_(op[:m])

        return self._issue(run, (out, inp), async_op)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        W = self.world
        if out.numel() != W * inp.numel() or inp.dtype != out.dtype:
            raise ValueError("all_gather: output must hold world x input elements of one dtype")
        v = self._vec(inp.dtype)

        def run():
            if self._fits(inp, v) and self._fits(out, v):
                self._ag(out, inp)
                return
            m = inp.numel()
            mp = -(-m // v) * v
            ip = torch.zeros(mp, dtype=inp.dtype, device=self.device)
            ip[:m].copy_(inp.reshape(-1))
            op = torch.empty(W, mp, dtype=out.dtype, device=self.device)
            self._ag(op.view(-1), ip)
            out.view(W, m).copy_(op[:, :m])

        return self._issue(run, (out, inp), async_op)

    def all_reduce(self, t: torch.Tensor, async_op: bool = False):
        """Two-shot all-reduce: reduce-scatter into a chunk, all-gather back in place."""
        W = self.world
        v = self._vec(t.dtype)

        def run():
            n = t.numel()
            m = -(-n // (W * v)) * v  # chunk per rank, a multiple of the vector
            if self._fits(t, v):
                part = torch.empty(m, dtype=t.dtype, device=self.device)
                self._rs(part, t.view(-1))
                self._ag(t.view(-1), part)
                return
            buf = torch.zeros(m * W, dtype=t.dtype, device=self.device)
            buf[:n].copy_(t.reshape(-1))
            part = torch.empty(m, dtype=t.dtype, device=self.device)
            self._rs(part, buf)
            self._ag(buf, part)
            t.copy_(buf[:n].view_as(t))

        return self._issue(run, (t,), async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        """Rank ``src``'s values everywhere (init-time only): an all-reduce of the source's
        tensor and zeros elsewhere."""
        if self.rank != src:
            t.zero_()
        self.all_reduce(t)

    def check(self):
        """Raise if any collective so far timed out.  Non-blocking: it sees a timeout of a
        collective that has already RUN; ``sync_check`` first waits for the last one."""
        if self._broken or self._c.error():
            self._broken = True
            raise RuntimeError("peer-memory collective timed out waiting for a peer (MXLLM_PEER_TIMEOUT_S); "
                               "the communicator is broken and its outputs since then are NaN")

    def sync_check(self):
        """Host-wait for the last collective issued, then ``check``: called before the optimizer
        consumes reduced gradients (DDP / ZeRO-1 ``finish``, ZeRO-3's step), so a timed-out
        exchange stops training with an error instead of feeding AdamW or a checkpoint."""
        if self._last is not None:
            self._last.synchronize()
        self.check()

    def close(self):
        try:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        finally:
            self._c.close()


def verify(*comms) -> None:
    """Before state is updated from collective results: for every peer-memory communicator
    among ``comms``, wait for its last collective and raise if a peer timed out.
    RCCL / gloo communicators report their own failures (watchdog / exceptions): no-op.
    ``MXLLM_PEER_SYNC_CHECK=0`` skips the host wait (the error then surfaces at a later wait)."""
    if os.environ.get("MXLLM_PEER_SYNC_CHECK", "1") == "0":
        return
    seen = set()
    for c in comms:
        f = getattr(c, "sync_check", None)
        if f is not None and id(c) not in seen:
            seen.add(id(c))
            f()


def peer_eligible(group=None, device: torch.device | None = None) -> bool:
    """Peer memory needs every rank of the group on this host and on a GPU."""
    if not dist.is_initialized() or device is None or device.type != "cuda":
        return False
    world = dist.get_world_size(group)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return 1 < world <= 16 and local_world >= dist.get_world_size()


def create_peer(group=None, device: torch.device | None = None, **kw) -> PeerCollectives | None:
    """Collective over ``group``: a :class:`PeerCollectives` on every rank, or None on every
    rank (never a mix: any local failure makes all ranks fall back)."""
    world = dist.get_world_size(group)
    comm, handle = None, None
    try:
        comm = PeerCollectives(group, device, **kw)
        handle = comm.handle()
    except Exception as e:  # noqa: BLE001
        log.warning("peer-memory communicator: local setup failed (%s)", e)
    handles: list = [None] * world
    dist.all_gather_object(handles, handle, group=group)
    ok = all(h is not None for h in handles)
    if ok:
        try:
            comm.open(handles)
            ok = comm.self_test()
        except Exception as e:  # noqa: BLE001
            log.warning("peer-memory communicator: opening peer buffers failed (%s)", e)
            ok = False
    oks: list = [None] * world
    dist.all_gather_object(oks, ok, group=group)
    if not all(oks):
        if comm is not None:
            comm.close()
        return None
    return comm


def create(group=None, device: torch.device | None = None, kind: str | None = None):
    """The communicator a trainer uses for ``group``.  Collective over ``group`` when the
    peer path is requested (``MXLLM_COMM=peer``); falls back to torch.distributed on every
    rank when peer memory is unusable (``MXLLM_COMM_STRICT=1``: raise instead)."""
    kind = kind or kind_requested()
    if kind == "peer" and dist.is_initialized() and dist.get_world_size(group) > 1:
        if peer_eligible(group, device):
            c = create_peer(group, device)
            if c is not None:
                log.info("[rank %d] bulk collectives: peer memory (world %d, %s schedule)", c.rank, c.world, c.algo)
                return c
        if os.environ.get("MXLLM_COMM_STRICT", "0") == "1":
            raise RuntimeError("MXLLM_COMM=peer requested but peer memory is unusable here")
        log.warning("MXLLM_COMM=peer unusable here; bulk collectives use torch.distributed")
    return TorchCollectives(group)
