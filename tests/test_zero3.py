"""ZeRO-3 correctness on CPU (gloo).

* per-parameter equality: after 3 optimizer steps (each rank its own batch,
  grad clipping + weight decay on) every fp32 master weight of the sharded
  trainer equals the replicated DDP trainer's, at world 1, 2 and 4, with and
  without activation checkpointing (every layer, or the first 2 of 3: selective);
* the loss trace matches too;
* the world-N emulation (one process, world-N shard sizes) runs and holds
  1/N of the optimizer state.
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


def _run(rank, world, port, q, mode, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.parallel.zero3 import Zero3Trainer
    from mxllm.train.trainer import OptimConfig, Trainer

    env = runtime.init(rank=rank, world_size=world)
    import mxllm.ops as mops

    recomputed = []  # selective checkpointing: the un-checkpointed layer recomputes m = swiglu(gu)
    _swl = mops.swiglu_linear
    mops.swiglu_linear = lambda *a: (recomputed.append(1), _swl(*a))[1]
    # "..._bf16": bf16 gradient reduction in both trainers (default: fp32 in both)
    gdt = torch.bfloat16 if mode.endswith("_bf16") else torch.float32
    mode = mode.removesuffix("_bf16")
    acc2 = mode.endswith("_acc2")  # two micro-batches per step (gradient accumulation)
    mode = mode.removesuffix("_acc2")
    cfg = get_config("tiny").replace(n_layers=3, vocab_size=320)
    opt = OptimConfig(lr=3e-3, grad_clip=1.0, weight_decay=0.01)
    if mode.startswith("zero3"):
        # "zero3_ckpt" = every layer checkpointed, "zero3_ckpt2" = the first 2 of 3 (selective)
        ck = mode.split("_ckpt")[1] if "_ckpt" in mode else None
        tr = Zero3Trainer(cfg, env, opt, seed=7, activation_checkpointing=(int(ck) if ck else True) if ck is not None
                          else False, grad_dtype=gdt)
    else:  # replicated DDP from the identical per-unit seeded init
        from mxllm.parallel.zero3 import init_full_state

        model = Llama(cfg, seed=0)
        sd = init_full_state(cfg, 7, env.device)
        with torch.no_grad():
            for n, p in model.named_parameters():
                p.copy_(sd[n])
        tr = Trainer(model, env, opt, grad_dtype=gdt)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (world * 2, 24), generator=g)
    losses = []
    mine = ids.view(world, 2, 24)[rank]  # fixed batch: the loss must go down
    mbs = [(mine[:1], mine[:1]), (mine[1:], mine[1:])] if acc2 else [(mine, mine)]
    for s in range(steps):
        losses.append(float(tr.train_step(mbs)))
    if mode == "zero3_ckpt2":
        assert len(recomputed) == steps * len(mbs), recomputed
    elif mode in ("zero3", "zero3_ckpt"):
        assert not recomputed
    if mode.startswith("zero3") and world > 1:
        # the default runs gathers and reduce-scatters on two communicators (split RCCL streams)
        assert tr.comm.rs_pg is not None and tr.comm.rs_pg is not tr.comm.ag_pg
    tot = runtime.all_reduce_scalars(losses, "sum")
    if mode.startswith("zero3"):
        master = tr.full_master_state()
    else:
        master = {s.name: tr.flat.master[s.offset:s.offset + s.numel].view(s.shape).clone() for s in tr.flat.slots}
    if rank == 0:
        q.put(([t / world for t in tot], {k: v.float().numpy().copy() for k, v in master.items()}))
    runtime.cleanup()


def _launch(mode, world, steps=3):
    import queue as _q
    import time

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_run, args=(r, world, port, q, mode, steps)) for r in range(world)]
    for p in ps:
        p.start()
    deadline = time.time() + 300
    while True:
        try:
            res = q.get(timeout=2)
            break
        except _q.Empty:
            assert not any(p.exitcode not in (None, 0) for p in ps), f"{mode} worker crashed"
            assert time.time() < deadline, "timeout"
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,gd", [(1, ""), (2, ""), (4, ""), (2, "_bf16"), (8, "_acc2")])
def test_zero3_matches_ddp_per_parameter(world, gd):
    """world 8 (BASELINE config 4's world) with gradient accumulation 2: plain and
    selective checkpointing (first 2 of 3 layers), split gather / reduce-scatter communicators."""
    ddp_loss, ddp_w = _launch("ddp" + gd, world)
    modes = {1: ["zero3", "zero3_ckpt", "zero3_ckpt2"], 2: ["zero3", "zero3_ckpt2"],
             8: ["zero3", "zero3_ckpt2"]}.get(world, ["zero3", "zero3_ckpt"])
    if gd == "_bf16":
        modes = ["zero3"]
    got = {}
    for mode in modes:
        z_loss, z_w = _launch(mode + gd, world)
        got[mode] = z_w
        assert ddp_loss[-1] < ddp_loss[0]  # it trains
        for x, y in zip(ddp_loss, z_loss):
            assert abs(x - y) < 2e-3 * max(1.0, abs(x)), (mode, ddp_loss, z_loss)
        assert set(ddp_w) == set(z_w)
        for n, w in ddp_w.items():
            # 3 AdamW steps of lr 3e-3 move a weight by up to ~1e-2; the replicas may differ
            # only by gradient summation order (all-reduce vs reduce-scatter): an element
            # whose summed gradient is ~0 can flip sign, moving by up to 2 lr per step
            d = abs(w - z_w[n])
            if world == 1:
                assert float(d.max()) < 1e-3, (mode, n, float(d.max()))  # CPU bf16 GEMM rounding only
            bad = int((d > 1e-3).sum())
            assert bad <= max(4, 5e-3 * d.size) and float(d.mean()) < 1e-4, (mode, n, bad, float(d.max()))
    for ck in ("zero3_ckpt", "zero3_ckpt2"):  # checkpointing recomputes the identical forward: bitwise equal
        if ck in got:
            for n, w in got["zero3"].items():
                assert (w == got[ck][n]).all(), (ck, n)


def test_zero3_emulated_world_shards():
    os.environ["MXLLM_FORCE_CPU"] = "1"
    from mxllm.models import get_config
    from mxllm.parallel.runtime import DistEnv
    from mxllm.parallel.zero3 import Zero3Trainer
    from mxllm.train.trainer import OptimConfig

    cfg = get_config("tiny").replace(n_layers=2, vocab_size=320)
    env = DistEnv()
    z1 = Zero3Trainer(cfg, env, OptimConfig(lr=1e-3), seed=3)
    z4 = Zero3Trainer(cfg, env, OptimConfig(lr=1e-3), seed=3, emulate_world=4, activation_checkpointing=True)
    assert z4.world == 4 and z4.emulated
    # sharded units hold 1/4 of their content; the replicated RMSNorm unit all of it
    assert z4.units[0].replicated and not any(u.replicated for u in z4.units[1:])
    assert z4.master.numel() == sum(u.full_numel // (1 if u.replicated else 4) for u in z4.units)
    assert z4.master.numel() < z1.master.numel() // 3
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    for _ in range(2):
        loss = z4.train_step([(ids, ids)])
    assert torch.isfinite(loss).all()


def test_rs_bf16_wire_emulated(monkeypatch):
    """MXLLM_Z3_RS_WIRE=bf16 (VERDICT r5 Missing 4): the emulated reduce-scatter stand-in sums the
    bf16-rounded contributions in fp32 and the link-byte account halves; fp32 stays exact."""
    from mxllm.parallel.zero3 import Comm

    full = torch.randn(4 * 1000, generator=torch.Generator().manual_seed(1))
    for wire in ("fp32", "bf16"):
        monkeypatch.setenv("MXLLM_Z3_RS_WIRE", wire)
        c = Comm(4, 0, emulate=4)
        out = torch.empty(1000)
        c.reduce_scatter(out, full, async_op=False)
        src = full.view(4, -1) if wire == "fp32" else full.view(4, -1).to(torch.bfloat16).float()
        assert torch.equal(out, src.sum(0))
        assert c.sent_bytes["rs"] == 3 * 1000 * (4 if wire == "fp32" else 2)
    monkeypatch.setenv("MXLLM_Z3_RS_WIRE", "fp16")
    with pytest.raises(ValueError):
        Comm(4, 0, emulate=4)
