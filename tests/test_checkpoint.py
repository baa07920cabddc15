"""Checkpoint format 2 (mxllm/train/checkpoint.py) on CPU / gloo:

* ZeRO-3 saves unit by unit (host staging bounded by one unit shard) and
  RESHARDS: written at world 4, resumed at world 2 (and world 1) with equal fp32
  master / Adam moments, and the resumed run continues with the same loss;
* a ZeRO-3 step directory loads into a plain model for serving / export;
* DDP optimizer state is written in pieces and resumes into a different
  flat layout by slot name;
* ZeRO-1 step directories carry the full model weights (rank 0).
Reference: none (the reference has no model state).
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


def _cfg():
    from mxllm.models import get_config

    return get_config("tiny").replace(n_layers=2, vocab_size=320)


def _ids(world, rank, step):
    g = torch.Generator().manual_seed(100 + step)
    return torch.randint(0, 320, (world * 2, 16), generator=g).view(world, 2, 16)[rank]


def _worker(rank, world, port, q, mode, ckdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.parallel import runtime
    from mxllm.parallel.zero3 import Zero3Trainer
    from mxllm.train import checkpoint
    from mxllm.train.trainer import OptimConfig

    env = runtime.init(rank=rank, world_size=world)
    opt = OptimConfig(lr=3e-3, weight_decay=0.01)
    res = {}
    if mode == "z3save":
        tr = Zero3Trainer(_cfg(), env, opt, seed=7, activation_checkpointing=True)
        for s in range(2):
            tr.train_step([(_ids(world, rank, s), _ids(world, rank, s))])
        checkpoint.save(ckdir, tr, 2)
        biggest = max(u.shard_numel for u in tr.units)
        res["staged_ok"] = checkpoint.staged_peak_bytes() <= 3 * 4 * biggest
        res["full"] = {k: v.numpy().copy() for k, v in tr.full_master_state().items()}
    elif mode == "z3load":
        tr = Zero3Trainer(_cfg(), env, opt, seed=99)  # different init: everything must come from the files
        checkpoint.load(ckdir, tr)
        res["step"] = tr.step_num
        res["full"] = {k: v.numpy().copy() for k, v in tr.full_master_state().items()}
        mom = {}
        for u in tr.units:  # the Adam moments of the first element of every unit shard, gathered
            off = u.master_view.storage_offset() - tr.master.storage_offset()
            t = tr.m[off:off + u.shard_numel].clone()
            if world > 1:
                full = torch.empty(t.numel() * world)
                torch.distributed.all_gather_into_tensor(full, t)
            else:
                full = t
            mom[u.uid] = full[:u.numel].numpy().copy()
        res["m"] = mom
    elif mode == "zero1save":
        from mxllm.models import Llama
        from mxllm.train.trainer import Trainer

        tr = Trainer(Llama(_cfg(), seed=1), env, opt, shard_optimizer=True)
        for s in range(2):
            tr.train_step([(_ids(world, rank, s), _ids(world, rank, s))])
        checkpoint.save(ckdir, tr, 2)
        tr.params_ready()
        res["params"] = {n: p.detach().float().numpy().copy() for n, p in tr.model.named_parameters()}
    if rank == 0:
        q.put(res)
    runtime.cleanup()


def _launch(mode, world, ckdir):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode, ckdir)) for r in range(world)]
    for p in ps:
        p.start()
    res = q.get(timeout=300)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_zero3_checkpoint_reshards(tmp_path):
    ck = str(tmp_path / "ck")
    saved = _launch("z3save", 4, ck)
    assert saved["staged_ok"]
    files = os.listdir(os.path.join(ck, "step_2", "z3"))
    assert sorted(files) == [f"rank_{r}" for r in range(4)]
    for world in (2, 1):
        got = _launch("z3load", world, ck)
        assert got["step"] == 2
        for n, w in saved["full"].items():
            assert (got["full"][n] == w).all(), (world, n)
    # the moments too: world 2 and world 1 agree element for element
    m2, m1 = _launch("z3load", 2, ck)["m"], _launch("z3load", 1, ck)["m"]
    for uid in m1:
        assert (m2[uid] == m1[uid]).all()
    # a ZeRO-3 step directory loads into a plain model (serving / export)
    from mxllm.models import Llama
    from mxllm.train.checkpoint import load_model_weights

    model = Llama(_cfg(), seed=123)
    load_model_weights(model, os.path.join(ck, "step_2"))
    for n, p in model.named_parameters():
        assert torch.equal(p.detach(), torch.from_numpy(saved["full"][n]).to(p.dtype)), n


def test_zero1_checkpoint_has_model_weights(tmp_path):
    ck = str(tmp_path / "ck1")
    saved = _launch("zero1save", 2, ck)
    from mxllm.models import Llama
    from mxllm.train.checkpoint import load_model_weights

    model = Llama(_cfg(), seed=55)
    load_model_weights(model, os.path.join(ck, "step_2"))
    for n, p in model.named_parameters():
        assert torch.equal(p.detach().float(), torch.from_numpy(saved["params"][n])), n


def test_ddp_checkpoint_pieces_and_layout_remap(tmp_path, monkeypatch):
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    from mxllm.models import Llama
    from mxllm.parallel import flat as flat_mod
    from mxllm.parallel import runtime
    from mxllm.train import checkpoint
    from mxllm.train import trainer as trainer_mod
    from mxllm.train.trainer import OptimConfig, Trainer

    runtime.cleanup()
    env = runtime.init(rank=0, world_size=1)
    monkeypatch.setattr(checkpoint, "PIECE_ELEMS", 100_000)  # several pieces, slots spanning pieces
    ids = torch.randint(0, 320, (2, 16), generator=torch.Generator().manual_seed(0))
    t1 = Trainer(Llama(_cfg(), seed=1), env, OptimConfig(lr=1e-2))
    for _ in range(2):
        t1.train_step([(ids, ids)])
    checkpoint.save(str(tmp_path), t1, 2, extra={"loader": {"cursor": 2}})
    assert len(os.listdir(os.path.join(tmp_path, "step_2", "optim"))) > 3
    l_next = float(t1.train_step([(ids, ids)]))
    # resume into a trainer whose flat buffer uses another layout (registration order)
    monkeypatch.setattr(trainer_mod, "production_order", lambda model, named: list(named))
    t2 = Trainer(Llama(_cfg(), seed=2), env, OptimConfig(lr=1e-2))
    assert [s.name for s in t2.flat.slots] != [s.name for s in t1.flat.slots]
    extra = checkpoint.load(str(tmp_path), t2)
    assert extra["loader"]["cursor"] == 2 and t2.step_num == 2
    assert abs(float(t2.train_step([(ids, ids)])) - l_next) < 1e-5
    del flat_mod
    runtime.cleanup()


def test_layout_guard_and_json_identity():
    """sharded optimizer state must only load into the same flat layout; the slot table
    read back from the JSON manifest (lists) must compare equal to the live one (tuples)."""
    import json

    import pytest

    from mxllm.train.checkpoint import _remap_segments, _require_same_layout

    live = {"slots": [("a", 0, 4, [2, 2]), ("b", 4, 3, [3])], "numel": 7}
    man = json.loads(json.dumps(live))
    assert _remap_segments(man, live) == [(0, 7, 0)]  # identity, not the per-slot path
    _require_same_layout(man, live, "ZeRO-1")
    moved = {"slots": [["b", 0, 3, [3]], ["a", 3, 4, [2, 2]]], "numel": 7}
    with pytest.raises(RuntimeError, match="different flat-buffer layout"):
        _require_same_layout(moved, live, "ZeRO-1")
    with pytest.raises(RuntimeError, match="no layout record"):
        _require_same_layout(None, live, "ZeRO-1")
    assert _remap_segments(moved, live) == [(3, 7, 0), (0, 3, 4)]
