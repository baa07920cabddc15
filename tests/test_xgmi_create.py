"""xGMI peer-memory communicator setup is all-or-nothing across ranks
(mxllm/parallel/xgmi.py ``create``): when ONE rank fails its local setup, or
one rank's peer-buffer open / self-test fails, EVERY rank gets None (and falls
back to RCCL) — never a mix, and no hang.  CPU / gloo with a stand-in
communicator class (the real one needs GPUs with IPC)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeComm:
    fail_init = -1
    fail_test = -1
    closed = False

    def __init__(self, rank, world, device):
        if rank == _FakeComm.fail_init:
            raise RuntimeError("injected: hipIpcGetMemHandle failed")
        self.rank = rank

    def handle(self):
        return f"handle-{self.rank}".encode()

    def open(self, handles):
        assert len(handles) >= 2 and all(h is not None for h in handles)

    def self_test(self):
        return self.rank != _FakeComm.fail_test

    def close(self):
        _FakeComm.closed = True


def _worker(rank, world, port, q, fail_init, fail_test):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    from mxllm.parallel import runtime, xgmi

    runtime.init(rank=rank, world_size=world)
    xgmi.eligible = lambda group=None: True  # the real check requires GPUs
    _FakeComm.fail_init, _FakeComm.fail_test = fail_init, fail_test
    comm = xgmi.create(None, cls=_FakeComm)
    q.put((rank, comm is None, _FakeComm.closed))
    runtime.cleanup()


@pytest.mark.parametrize("world,fail_init,fail_test", [(2, 1, -1), (4, 2, -1), (4, -1, 0), (2, -1, -1)])
def test_create_is_all_or_nothing(world, fail_init, fail_test):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, fail_init, fail_test)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    none = {r: n for r, n, _ in res}
    expect_none = fail_init >= 0 or fail_test >= 0
    assert all(v == expect_none for v in none.values()), none
    if fail_test >= 0:  # ranks that had opened their buffers closed them again
        assert all(c for r, n, c in res)
