"""Context parallelism (ring attention, zigzag layout; mxllm/parallel/context.py)
on CPU / gloo: P ranks each hold 2 of the 2P chunks of every sequence; the
world-averaged loss and DDP-averaged gradients equal the single-process model
on the full sequence (P = 2 and 4, GQA tiny model)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg():
    from mxllm.models import get_config

    return get_config("tiny").replace(n_layers=2, vocab_size=300)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    import torch.distributed as dist

    from mxllm.models import Llama
    from mxllm.parallel import runtime
    from mxllm.parallel.context import zigzag_shard
    from mxllm.parallel.sequence import new_groups
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    cfg = _cfg()
    model = Llama(cfg, lora_r=0, seed=3).float()
    grp, dp_rank, dp_world = new_groups(world)
    model.set_context_parallel(grp)
    tr = Trainer(model, env, OptimConfig(lr=1e-2, grad_clip=0.0))
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    lab = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    loss = model(zigzag_shard(ids, grp), zigzag_shard(lab, grp))
    loss.backward()
    scale = tr.ddp.finish()
    grads = (tr.flat.grads.clone() * scale).numpy()
    lsum = loss.detach().clone()
    dist.all_reduce(lsum)
    if rank == 0:
        q.put((float(lsum) / world, grads))
    runtime.cleanup()


def test_zigzag_shard_roundtrip():
    from mxllm.parallel.context import zigzag_positions, zigzag_unshard

    P, S = 4, 64
    t = torch.arange(S).view(1, S)
    C = S // (2 * P)
    parts = [torch.cat([t[:, r * C:(r + 1) * C], t[:, (2 * P - 1 - r) * C:(2 * P - r) * C]], 1) for r in range(P)]
    assert torch.equal(zigzag_unshard(parts), t)
    for r in range(P):
        assert torch.equal(zigzag_positions(S // P, P, r), parts[r][0])


@pytest.mark.parametrize("world", [2, 4])
def test_ring_attention_matches_full_sequence(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    loss_cp, grads_cp = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0

    from mxllm.models import Llama
    from mxllm.parallel.flat import FlatParams, production_order

    cfg = _cfg()
    model = Llama(cfg, lora_r=0, seed=3).float()
    flat = FlatParams(production_order(model, [(n, p) for n, p in model.named_parameters() if p.requires_grad]),
                      reverse=False)  # the Trainer's layout
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    lab = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    loss = model(ids, lab)
    loss.backward()
    flat.sync_grads_from_params()
    assert abs(float(loss) - loss_cp) < 1e-4, (float(loss), loss_cp)
    torch.testing.assert_close(torch.from_numpy(grads_cp), flat.grads, rtol=2e-3, atol=2e-5)
