"""Process-group runtime: torchrun env contract, device binding, RCCL/gloo.

Reference behaviour (src/distributed_inference.py:14-21, 46-51) and the fixes
SURVEY §0.4 requires:
  * D3 — torchrun-provided MASTER_ADDR/MASTER_PORT are never overwritten; a
    CONFIG value is only used when the launcher did not provide one.
  * D4 — every process binds ``cuda:LOCAL_RANK`` before creating the group
    (one process per GPU), and passes ``device_id`` so RCCL binds eagerly.
  * D6 — ``cleanup()`` is idempotent and safe on error paths.
  * D7 — backend chosen from device availability: ``nccl`` (= RCCL over xGMI
    on ROCm) with GPUs, ``gloo`` on CPU; explicit timeouts everywhere.
"""
from __future__ import annotations

import datetime
import logging
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

log = logging.getLogger("mxllm.dist")


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_rank: int = 0
    backend: str = "gloo"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_ENV: DistEnv | None = None
_SMALL = None  # XgmiComm for latency-bound collectives (xgmi.py), when usable


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def gpu_available() -> bool:
    return torch.cuda.is_available() and os.environ.get("MXLLM_FORCE_CPU") != "1"


def pick_device(local_rank: int) -> torch.device:
    if gpu_available():
        n = torch.cuda.device_count()
        idx = local_rank % max(n, 1)
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    return torch.device("cpu")


def init(backend: str | None = None, timeout_s: float | None = None, rank: int | None = None,
         world_size: int | None = None, master_addr: str | None = None, master_port: int | str | None = None,
         barrier: bool = True) -> DistEnv:
    """Initialise (or return) the process group from the torchrun environment.

    ``rank``/``world_size`` override env (the reference's ``setup(rank, world)``
    signature); ``master_addr``/``master_port`` are defaults used only when the
    launcher did not export them.
    """
    global _ENV
    if _ENV is not None and (dist.is_initialized() or _ENV.world_size == 1):
        return _ENV
    rank = env_int("RANK", 0) if rank is None else rank
    world_size = env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = env_int("LOCAL_RANK", rank if world_size <= env_int("LOCAL_WORLD_SIZE", world_size) else 0)
    local_world = env_int("LOCAL_WORLD_SIZE", world_size)
    node_rank = env_int("GROUP_RANK", env_int("NODE_RANK", 0))
    device = pick_device(local_rank)
    if backend is None:
        backend = os.environ.get("MXLLM_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
    e = DistEnv(rank, world_size, local_rank, local_world, node_rank, backend, device)
    if world_size > 1 and not dist.is_initialized():
        if "MASTER_ADDR" not in os.environ:
            os.environ["MASTER_ADDR"] = str(master_addr or "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(master_port or 29500)
        if timeout_s is None:
            timeout_s = float(os.environ.get("MXLLM_PG_TIMEOUT_S", "600"))
        kw = dict(backend=backend, rank=rank, world_size=world_size,
                  timeout=datetime.timedelta(seconds=timeout_s), store=_attempt_store(rank, world_size, timeout_s))
        if backend == "nccl" and device.type == "cuda":
            kw["device_id"] = device
        dist.init_process_group(**kw)
        log.debug("[rank %d] process group up: backend=%s world=%d device=%s", rank, backend, world_size, device)
        if barrier:
            if backend == "nccl":
                dist.barrier(device_ids=[device.index])
            else:
                dist.barrier()
        if backend == "nccl" and device.type == "cuda":
            global _SMALL
            from . import xgmi

            _SMALL = xgmi.create(device)
            log.debug("[rank %d] small-message collectives: %s", rank, "xGMI peer memory" if _SMALL else "RCCL")
    _ENV = e
    return e


def small_comm():
    """The xGMI peer-memory communicator (or None: use torch.distributed)."""
    return _SMALL


def _attempt_store(rank: int, world_size: int, timeout_s: float):
    """TCPStore client (or rank-0 server when not under torchrun) namespaced by
    the elastic restart attempt: after ``--max-restarts`` the agent keeps its
    store, and without a per-attempt prefix restarted ranks would read the dead
    attempt's rendezvous keys (stale peer addresses) and fail to connect."""
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world_size=world_size,
                          is_master=(not agent and rank == 0), timeout=datetime.timedelta(seconds=timeout_s),
                          wait_for_workers=False)
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return dist.PrefixStore(f"mxllm/attempt_{attempt}", store)


def get_env() -> DistEnv:
    return _ENV if _ENV is not None else init()


def cleanup() -> None:
    """Destroy the process group if one exists (idempotent)."""
    global _ENV, _SMALL
    if _SMALL is not None:
        try:
            _SMALL.close()
        except Exception as e:  # noqa: BLE001
            log.warning("closing xGMI communicator failed: %s", e)
        _SMALL = None
    if dist.is_available() and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001
            log.warning("destroy_process_group failed: %s", e)
    _ENV = None


def barrier() -> None:
    if dist.is_initialized():
        e = get_env()
        if e.backend == "nccl":
            dist.barrier(device_ids=[e.device.index])
        else:
            dist.barrier()


def all_reduce_scalars(vals: list[float], op: str = "sum", device=None) -> list[float]:
    """Reduce a handful of host scalars across ranks in one collective."""
    if not dist.is_initialized():
        return list(vals)
    e = get_env()
    if _SMALL is not None and len(vals) <= _SMALL.max_elems:
        t = torch.tensor(vals, dtype=torch.float32, device=e.device)
        _SMALL.all_reduce_(t, op)
        out = t.tolist()
        _SMALL.check()
        return out
    t = torch.tensor(vals, dtype=torch.float64 if e.backend == "gloo" else torch.float32,
                     device=device or e.device)
    dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return t.tolist()


def all_reduce_small_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce of a small device tensor without a host sync
    (xGMI one-shot kernel when available, else torch.distributed)."""
    if not dist.is_initialized():
        return t
    if (_SMALL is not None and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
            and t.numel() <= _SMALL.max_elems):
        return _SMALL.all_reduce_(t, op)
    dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return t


def all_gather_objects(obj) -> list:
    """Gather one picklable object per rank (rank order); ``[obj]`` without a process group."""
    if not dist.is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
