"""GEMM dispatch policy (mxllm/ops/gemm.py) on CPU: the measured-win table and the persistent-kernel
guard for multi-rank runs."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mxllm.ops import gemm


def _persistent_entry():
    for key, ph in gemm._table().items():
        if ph == 5:
            return key
    pytest.skip("no persistent (ph 5) entry in the tuning table")


def test_table_has_persistent_fp32_dw_entries():
    form, M, N, K, out = _persistent_entry()
    assert form == "tt" and out == "f32"
    assert gemm.schedule(form, M, N, K, torch.float32) == 5  # world 1: the persistent kernel


def _worker(rank, world, port, key, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mxllm.ops import gemm as g

    form, M, N, K, _ = key
    q.put((rank, g.schedule(form, M, N, K, torch.float32)))
    dist.destroy_process_group()


def test_persistent_gemm_is_world1_only():
    """In a group of > 1 ranks the persistent shapes fall back to the one-tile-per-workgroup 4-phase
    launch (collective kernels holding CUs would stall the fixed tile shares)."""
    key = _persistent_entry()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, key, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert got == {0: 4, 1: 4}
