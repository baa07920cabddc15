"""Tensor-parallel serving (mxllm/parallel/tensor.py) on CPU: gloo, spawned ranks.

The TP=2 / TP=4 shards of a model, run through the engine with the group's
all-reduces and vocab-parallel head, must reproduce the single-process engine:
same prefill logits (fp32 model, so only summation order differs) and the same
greedy tokens; every rank sees identical logits.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    from mxllm.models import Llama, get_config

    cfg = get_config("tiny").replace(n_layers=2, vocab_size=301, n_heads=8, n_kv_heads=4, ffn=256)
    return Llama(cfg, dtype=torch.float32, seed=5).eval()


PROMPTS = [[1, 5, 9, 13, 200], [7, 7, 3], [250, 11, 42, 42, 17, 99, 3]]


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    import torch.distributed as dist

    from mxllm.parallel import runtime
    from mxllm.parallel.tensor import shard_llama
    from mxllm.serve.engine import Engine

    runtime.init(rank=rank, world_size=world)
    full = _model()
    local = shard_llama(full, rank, world)
    del full
    eng = Engine(local, max_batch=4, max_seq=64, tp_group=dist.group.WORLD)
    logits = eng.prefill_batch([0, 1, 2], PROMPTS)
    eng.lens = [0] * 4
    outs = Engine(local, max_batch=4, max_seq=64, tp_group=dist.group.WORLD).generate(PROMPTS, max_new_tokens=6)
    all_logits = [torch.zeros_like(logits) for _ in range(world)]
    dist.all_gather(all_logits, logits)
    same = all(torch.equal(all_logits[0], x) for x in all_logits)
    if rank == 0:
        out_q.put((logits, outs, same, local.cfg.n_heads, local.lm_head.shape[0]))
    runtime.cleanup()


@pytest.mark.parametrize("world", [2, 4])
def test_tp_engine_matches_single_process(world):
    from mxllm.serve.engine import Engine

    full = _model()
    eng = Engine(full, max_batch=4, max_seq=64)
    ref_logits = eng.prefill_batch([0, 1, 2], PROMPTS)
    ref_out = Engine(full, max_batch=4, max_seq=64).generate(PROMPTS, max_new_tokens=6)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    logits, outs, same, nh, vrows = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert same, "ranks disagree on the gathered logits"
    assert nh == 8 // world and vrows * world >= 301
    assert logits.shape == ref_logits.shape
    assert torch.allclose(logits, ref_logits, atol=1e-4, rtol=1e-4), (logits - ref_logits).abs().max()
    assert outs == ref_out


def test_shard_config_divisibility():
    from mxllm.models import get_config
    from mxllm.parallel.tensor import shard_config, vocab_shard_rows

    c = shard_config(get_config("llama3.1-70b"), 8)
    assert (c.n_heads, c.n_kv_heads, c.ffn, c.hidden) == (8, 1, 3584, 8192)
    assert vocab_shard_rows(128256, 8) * 8 >= 128256
    with pytest.raises(ValueError):
        shard_config(get_config("llama3.1-70b"), 16)


def _server_worker(rank, world, port, out_q):
    """Server mode: only rank 0 receives requests (background engine loop, with
    idle heartbeats); rank 1 mirrors its schedule through ``follow()``."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    import time

    import torch.distributed as dist

    from mxllm.parallel import runtime
    from mxllm.parallel.tensor import shard_llama
    from mxllm.serve.engine import Engine, SamplingParams

    runtime.init(rank=rank, world_size=world)
    local = shard_llama(_model(), rank, world)
    eng = Engine(local, max_batch=2, max_seq=64, tp_group=dist.group.WORLD)
    eng.enable_tp_sync()
    if rank != 0:
        eng.follow()
        runtime.cleanup()
        return
    eng.start()
    time.sleep(1.2)  # idle: the followers are kept in step by heartbeats
    reqs = [eng.submit(p, SamplingParams(max_new_tokens=5)) for p in PROMPTS]  # 3 requests, 2 slots
    for r in reqs:
        assert r.done.wait(120)
    eng.stop()
    out_q.put([r.output for r in reqs])
    runtime.cleanup()


def test_tp_server_mode_follows_rank0():
    from mxllm.serve.engine import Engine

    ref_out = Engine(_model(), max_batch=2, max_seq=64).generate(PROMPTS, max_new_tokens=5)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_server_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert outs == ref_out
