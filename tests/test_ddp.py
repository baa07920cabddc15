"""Distributed correctness on CPU (gloo, spawned ranks) — SURVEY §4.2 item 5.

* mxllm DDP (flat buckets, async all-reduce from grad hooks) produces exactly
  the gradient of the single-process model on the concatenated batch;
* after one optimizer step every rank holds identical parameters;
* gradient accumulation with no_sync matches one big batch.
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


def _worker(rank, world, port, out_q, full, bucket_mb, accum):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    cfg = get_config("tiny").replace(n_layers=2, vocab_size=300)
    torch.manual_seed(0)
    model = Llama(cfg, lora_r=0 if full else 4, seed=3)
    if not full:  # make LoRA B non-zero so every adapter gets gradient
        with torch.no_grad():
            for i, mod in enumerate(model.modules()):
                if getattr(mod, "lora_r", 0):
                    for blk in mod.lora_b_blocks():
                        blk.normal_(0, 0.02, generator=torch.Generator().manual_seed(i))
    tr = Trainer(model, env, OptimConfig(lr=1e-2, grad_clip=0.0), bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, cfg.vocab_size, (world * 2 * accum, 32), generator=g)
    mine = ids.view(world, 2 * accum, 32)[rank]
    mbs = [(mine[i * 2:(i + 1) * 2], mine[i * 2:(i + 1) * 2]) for i in range(accum)]
    # grads after all-reduce (captured via a hook on finish)
    n = len(mbs)
    for i, (a, b) in enumerate(mbs):
        ctx = tr.ddp.no_sync() if i < n - 1 else torch.enable_grad()
        with ctx:
            (model(a, b) / n).backward()
    scale = tr.ddp.finish()
    grads = (tr.flat.grads.clone() * scale).tolist() if rank == 0 else None
    tr.flat.zero_grad()
    tr.train_step(mbs)
    params = tr.flat.params.clone()
    allp = [torch.zeros_like(params) for _ in range(world)]
    torch.distributed.all_gather(allp, params)
    same = all(torch.equal(allp[0], p) for p in allp)
    if rank == 0:
        out_q.put((grads, same, len(tr.ddp.buckets)))
    runtime.cleanup()


def _single_grads(world, full, accum):
    os.environ["MXLLM_FORCE_CPU"] = "1"
    from mxllm.models import Llama, get_config
    from mxllm.parallel.flat import FlatParams, production_order

    cfg = get_config("tiny").replace(n_layers=2, vocab_size=300)
    model = Llama(cfg, lora_r=0 if full else 4, seed=3)
    if not full:
        with torch.no_grad():
            for i, mod in enumerate(model.modules()):
                if getattr(mod, "lora_r", 0):
                    for blk in mod.lora_b_blocks():
                        blk.normal_(0, 0.02, generator=torch.Generator().manual_seed(i))
        model.sync_adapters_()
    flat = FlatParams(production_order(model, [(n, p) for n, p in model.named_parameters() if p.requires_grad]),
                      reverse=False)  # the Trainer's layout
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, cfg.vocab_size, (world * 2 * accum, 32), generator=g)
    # per-rank mean over micro-batches, then mean over ranks == mean over equal chunks
    total = 0
    for r in range(world):
        mine = ids.view(world, 2 * accum, 32)[r]
        for i in range(accum):
            total = total + model(mine[i * 2:(i + 1) * 2], mine[i * 2:(i + 1) * 2]) / (accum * world)
    total.backward()
    flat.sync_grads_from_params()
    return flat.grads.clone()


@pytest.mark.parametrize("full,bucket_mb,accum,world", [(True, 0.05, 1, 2), (False, 0.01, 1, 2), (True, 0.05, 2, 2),
                                                         (True, 0.05, 1, 4)])
def test_ddp_matches_single_process(full, bucket_mb, accum, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, full, bucket_mb, accum)) for r in range(world)]
    for p in procs:
        p.start()
    grads, same, nb = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref = _single_grads(world, full, accum)
    got = torch.tensor(grads, dtype=ref.dtype)
    assert nb > 1, "test should exercise multiple buckets"
    err = (got.float() - ref.float()).abs().max().item()
    tol = 2e-2 if ref.dtype == torch.bfloat16 else 1e-5
    assert err <= tol * max(1.0, ref.float().abs().max().item()), err
    assert same, "ranks diverged after the optimizer step"


def test_fresh_guard_zeroes_stale_slot_before_autograd_accumulates():
    """ADVICE r3 (fresh gradients): a parameter whose gradient arrives through autograd's
    AccumulateGrad while its flat slot is still flagged fresh must not be added onto last
    step's stale gradient: the guard hook zeroes the slot first, once."""
    from mxllm.train.trainer import _fresh_guard

    p = torch.nn.Parameter(torch.ones(4))
    p.grad = torch.full((4,), 7.0)  # stale slot content from the previous step
    p._mx_grad_fresh = True
    p.register_hook(_fresh_guard(p))
    ((p * 2).sum() + (p * 3).sum()).backward()  # two contributions: zero once, then both accumulate
    assert torch.equal(p.grad, torch.full((4,), 5.0))
    assert p._mx_grad_fresh is False


def test_grad_norm_under_accumulation_matches_one_batch(monkeypatch):
    """World 1: two micro-batches of 2 sequences clip on the same gradient norm as one
    micro-batch of the 4 (the flat buffer holds the micro-batch MEAN; the scale is 1/world)."""
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    from mxllm.models import Llama, get_config
    from mxllm.parallel.runtime import DistEnv
    from mxllm.train.trainer import OptimConfig, Trainer

    cfg = get_config("tiny").replace(n_layers=2, vocab_size=300)
    ids = torch.randint(0, cfg.vocab_size, (4, 32), generator=torch.Generator().manual_seed(3))
    norms = []
    for mbs in ([(ids, ids)], [(ids[:2], ids[:2]), (ids[2:], ids[2:])]):
        tr = Trainer(Llama(cfg, dtype=torch.float32, seed=5), DistEnv(), OptimConfig(lr=1e-3, grad_clip=1.0))
        tr.train_step(mbs)
        norms.append(float(tr.last_grad_norm))
    assert abs(norms[0] - norms[1]) < 1e-4 * norms[0], norms


def test_finish_runs_the_peer_sync_check(monkeypatch):
    """DDP.finish waits for a peer communicator's last collective and raises on a
    timeout BEFORE the optimizer consumes the reduced gradient (comm.verify); RCCL / gloo
    communicators have no such hook and pass through; MXLLM_PEER_SYNC_CHECK=0 skips it."""
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    from mxllm.models import Llama, get_config
    from mxllm.parallel.ddp import DDP
    from mxllm.parallel.flat import FlatParams, production_order

    class BrokenPeer:
        kind = "peer"
        checked = 0

        def all_reduce(self, t, async_op=False):
            return None

        def sync_check(self):
            BrokenPeer.checked += 1
            raise RuntimeError("peer-memory collective timed out")

    model = Llama(get_config("tiny").replace(n_layers=1, vocab_size=64), dtype=torch.float32, seed=1)
    flat = FlatParams(production_order(model, [(n, p) for n, p in model.named_parameters()]), reverse=False)
    ddp = DDP(flat, enabled=True, comm=BrokenPeer())
    with pytest.raises(RuntimeError, match="timed out"):
        ddp.finish()
    assert BrokenPeer.checked == 1
    monkeypatch.setenv("MXLLM_PEER_SYNC_CHECK", "0")
    assert ddp.finish() == 1.0  # world 1 scale; the check skipped
