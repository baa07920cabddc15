"""Ulysses sequence parallelism (mxllm/parallel/sequence.py) on CPU, gloo.

Two ranks each hold half of every sequence; attention runs on the full
sequence with half of the heads after an all-to-all.  The world-averaged loss
and DDP-averaged gradients must equal the single-process model on the full
sequence.
"""
import os
import socket

import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    import torch.distributed as dist

    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.parallel.sequence import new_groups, shard_sequence
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    cfg = get_config("tiny").replace(n_layers=2, vocab_size=300)
    model = Llama(cfg, lora_r=0, seed=3).float()
    grp, dp_rank, dp_world = new_groups(world)
    assert dp_world == 1
    model.set_sequence_parallel(grp)
    tr = Trainer(model, env, OptimConfig(lr=1e-2, grad_clip=0.0))
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    lab = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    loss = model(shard_sequence(ids, grp), shard_sequence(lab, grp))
    loss.backward()
    scale = tr.ddp.finish()
    grads = tr.flat.grads.clone() * scale
    lsum = loss.detach().clone()
    dist.all_reduce(lsum)
    if rank == 0:
        q.put((float(lsum) / world, grads))
    runtime.cleanup()


def test_ulysses_matches_full_sequence():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    loss_sp, grads_sp = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0

    from mxllm.models import Llama, get_config
    from mxllm.parallel.flat import FlatParams, production_order

    cfg = get_config("tiny").replace(n_layers=2, vocab_size=300)
    model = Llama(cfg, lora_r=0, seed=3).float()
    flat = FlatParams(production_order(model, [(n, p) for n, p in model.named_parameters() if p.requires_grad]),
                      reverse=False)  # the Trainer's layout
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    lab = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    loss = model(ids, lab)
    loss.backward()
    flat.sync_grads_from_params()
    assert abs(float(loss) - loss_sp) < 1e-4, (float(loss), loss_sp)
    torch.testing.assert_close(grads_sp, flat.grads, rtol=2e-3, atol=2e-5)
