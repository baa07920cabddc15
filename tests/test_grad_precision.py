"""Gradient-reduction precision (SURVEY §2.3 "flat bf16/fp32
buckets", C6 "fp32 accumulate option"; reference claim README.md:7).

gloo world 8 on CPU: every rank forms its micro-batch gradient and the bucketed
DDP all-reduce sums them.  The oracle is the fp64 sum of the same eight per-rank
fp32 gradients computed in ONE process.  With ``grad_dtype=float32`` the only
error left is the fp32 ring summation (asserted < 1e-6 relative); the bf16 path
rounds every local gradient and every partial sum to bf16.
"""
import os
import socket

import torch
import torch.multiprocessing as mp

WORLD = 8


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg():
    from mxllm.models import get_config

    return get_config("tiny").replace(n_layers=2, vocab_size=320)


def _batch(rank):
    g = torch.Generator().manual_seed(1000 + rank)
    ids = torch.randint(0, 320, (2, 32), generator=g)
    return ids, ids


def _trainer(env, gdt):
    from mxllm.models import Llama
    from mxllm.train.trainer import OptimConfig, Trainer

    return Trainer(Llama(_cfg(), seed=4), env, OptimConfig(), grad_dtype=gdt, overlap_optimizer=False)


def _worker(rank, port, q, gd):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.parallel import runtime

    env = runtime.init(rank=rank, world_size=WORLD)
    tr = _trainer(env, torch.float32 if gd == "fp32" else torch.bfloat16)
    tr.compute_grads([_batch(rank)])  # forward + backward + bucketed all-reduce (SUM)
    if rank == 0:
        q.put(tr.flat.grads.double().numpy().copy())
    runtime.cleanup()


def _reduced(gd):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q, gd)) for r in range(WORLD)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return torch.from_numpy(out)


def test_fp32_reduction_matches_fp64_oracle_world8(monkeypatch):
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    from mxllm.parallel.runtime import DistEnv

    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # the ranks' arithmetic, bit for bit
    try:
        oracle = None
        for r in range(WORLD):
            tr = _trainer(DistEnv(), torch.float32)
            tr.compute_grads([_batch(r)])
            g = tr.flat.grads.double()
            oracle = g if oracle is None else oracle + g
    finally:
        torch.set_num_threads(nt)
    err = {}
    for gd in ("fp32", "bf16"):
        got = _reduced(gd)
        err[gd] = ((got - oracle).norm() / oracle.norm()).item()
    print(f"relative error of the world-8 reduced gradient vs the fp64 oracle: {err}")
    assert err["fp32"] < 1e-6, err
    assert err["bf16"] > 10 * err["fp32"], err  # the bf16 path really rounds (and the test can tell)
