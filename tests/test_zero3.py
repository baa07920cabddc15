"""ZeRO-3 correctness on CPU (gloo): sharded training matches the replicated
DDP trainer step for step (same init, same data), world 1 and 2."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, q, mode, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.parallel.zero3 import Zero3Trainer
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    cfg = get_config("tiny").replace(n_layers=3, vocab_size=320)
    opt = OptimConfig(lr=3e-3, grad_clip=1.0, weight_decay=0.01)
    if mode == "zero3":
        tr = Zero3Trainer(cfg, env, opt, seed=7)
    else:  # replicated DDP from the identical per-unit seeded init
        from mxllm.parallel.zero3 import init_full_state

        model = Llama(cfg, seed=0)
        sd = init_full_state(cfg, 7, env.device)
        with torch.no_grad():
            for n, p in model.named_parameters():
                p.copy_(sd[n])
        tr = Trainer(model, env, opt)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (world * 2, 24), generator=g)
    losses = []
    mine = ids.view(world, 2, 24)[rank]  # fixed batch: the loss must go down
    for s in range(steps):
        losses.append(float(tr.train_step([(mine, mine)])))
    tot = runtime.all_reduce_scalars(losses, "sum")
    if rank == 0:
        q.put([t / world for t in tot])
    runtime.cleanup()


@pytest.mark.parametrize("world", [1, 2])
def test_zero3_matches_ddp(world):
    ctx = mp.get_context("spawn")
    res = {}
    for mode in ("ddp", "zero3"):
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_run, args=(r, world, port, q, mode, 4)) for r in range(world)]
        for p in ps:
            p.start()
        import queue as _q
        import time

        deadline = time.time() + 300
        while True:
            try:
                res[mode] = q.get(timeout=2)
                break
            except _q.Empty:
                assert not any(p.exitcode not in (None, 0) for p in ps), f"{mode} worker crashed"
                assert time.time() < deadline, "timeout"
        for p in ps:
            p.join(60)
            assert p.exitcode == 0
    a, b = res["ddp"], res["zero3"]
    assert a[-1] < a[0]  # it trains
    for x, y in zip(a, b):
        assert abs(x - y) < 2e-2 * max(1.0, abs(x)), (a, b)
