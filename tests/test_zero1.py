"""ZeRO-1 (sharded optimizer over reduce-scattered DDP buckets) on CPU / gloo.

After 3 optimizer steps (every rank its own batch, grad clipping and weight
decay on, several buckets) every fp32 master weight equals plain DDP's, all
ranks hold bitwise-identical bf16 parameters, and a DDP run at world 4 keeps
its replicas identical too.  Reference claim: DDP fine-tuning (README.md:7).
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


def _run(rank, world, port, q, shard, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    cfg = get_config("tiny").replace(n_layers=3, vocab_size=320)
    model = Llama(cfg, seed=11)
    tr = Trainer(model, env, OptimConfig(lr=3e-3, grad_clip=1.0, weight_decay=0.01), bucket_mb=0.2,
                 first_bucket_mb=0.05, shard_optimizer=shard)
    assert (tr.zero1 is not None) == shard
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (world * 2, 24), generator=g)
    mine = ids.view(world, 2, 24)[rank]
    losses = [float(tr.train_step([(mine, mine)])) for _ in range(steps)]
    if shard:
        tr.zero1.wait_params()
        master = tr.zero1.full_master()
    else:
        master = tr.flat.master.float().clone()
    params = tr.flat.params.clone()
    allp = [torch.zeros_like(params) for _ in range(world)]
    torch.distributed.all_gather(allp, params)
    same = all(torch.equal(allp[0], p) for p in allp)
    named = {s.name: master[s.offset:s.offset + s.numel].numpy().copy() for s in tr.flat.slots}
    if rank == 0:
        q.put((losses, named, same, len(tr.ddp.buckets)))
    runtime.cleanup()


def _launch(world, shard, steps=3):
    import queue as _q
    import time

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_run, args=(r, world, port, q, shard, steps)) for r in range(world)]
    for p in ps:
        p.start()
    deadline = time.time() + 300
    while True:
        try:
            res = q.get(timeout=2)
            break
        except _q.Empty:
            assert not any(p.exitcode not in (None, 0) for p in ps), "worker crashed"
            assert time.time() < deadline, "timeout"
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_zero1_matches_ddp_per_parameter(world):
    d_loss, d_w, d_same, nb = _launch(world, False)
    z_loss, z_w, z_same, _ = _launch(world, True)
    assert nb > 2, "several buckets expected"
    assert d_same and z_same, "replicas diverged"
    assert d_loss[-1] < d_loss[0]
    for x, y in zip(d_loss, z_loss):
        assert abs(x - y) < 2e-3 * max(1.0, abs(x)), (d_loss, z_loss)
    for n, w in d_w.items():
        d = abs(w - z_w[n])
        # bf16 gradient sums in a different order (all-reduce vs reduce-scatter) may flip
        # the sign of a ~0 gradient element: rare, bounded by 2 lr per step
        bad = int((d > 1e-3).sum())
        assert bad <= max(4, 5e-3 * d.size) and float(d.mean()) < 1e-4, (n, bad, float(d.max()))
