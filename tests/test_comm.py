"""Small-message collectives and the desync detector.

CPU: the parameter-checksum check over gloo (2 spawned ranks) accepts
identical replicas and names a perturbed one.
GPU: the xGMI one-shot all-reduce kernel (csrc/kernels/xgmi.hip) with two
processes sharing the box's one MI355X through IPC-mapped peer buffers —
the same code path as 8 GPUs on the xGMI mesh, minus the link hop: sum /
max / min against an fp64 host reference, uneven arrival (one rank sleeps),
a device barrier, and the bounded-spin timeout (NaN + error flag) when a
peer never arrives.
"""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# --------------------------------------------------------------------- CPU


def _sync_worker(rank, world, port, q, perturb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_FORCE_CPU="1")
    torch.set_num_threads(1)
    from mxllm.parallel import runtime
    from mxllm.parallel.consistency import check_in_sync

    runtime.init(rank=rank, world_size=world)
    p = torch.randn(10_000, generator=torch.Generator().manual_seed(0)).to(torch.bfloat16)
    if perturb and rank == 1:
        p[1234] = p[1234] + 1
    try:
        ok = check_in_sync([p, p.float()], raise_on_mismatch=False)
    finally:
        runtime.cleanup()
    q.put((rank, ok))


@pytest.mark.parametrize("perturb", [False, True])
def test_check_in_sync_two_ranks(perturb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_sync_worker, args=(r, 2, port, q, perturb)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: not perturb, 1: not perturb}


def test_param_checksum_sensitivity():
    from mxllm.parallel.consistency import param_checksum

    a = torch.arange(1000, dtype=torch.float32).to(torch.bfloat16)
    b = a.clone()
    assert param_checksum(a) == param_checksum(b)
    b[3], b[4] = a[4].clone(), a[3].clone()
    assert param_checksum(a) != param_checksum(b)
    c = a.clone()
    c.view(torch.int16)[10] ^= 1  # one flipped mantissa bit
    assert param_checksum(a) != param_checksum(c)


# --------------------------------------------------------------------- GPU


def _xgmi_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_XGMI="1")  # opt-in path
    import torch.distributed as dist

    from mxllm.parallel import xgmi

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"rank": rank}
    try:
        comm = xgmi.create(dev, timeout_s=30.0)
        out["created"] = comm is not None
        if comm is None:
            return
        errs = []
        for it in range(40):
            n = [1, 3, 64, 1000, 4096][it % 5]
            vals = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r), dtype=torch.float64)
                    for r in range(world)]
            op = ["sum", "max", "min"][it % 3]
            if rank == 1 and it % 4 == 1:
                time.sleep(0.05)  # uneven arrival: the peer's kernel spins on the flag
            t = vals[rank].to(torch.float32).to(dev)
            comm.all_reduce_(t, op)
            ref = vals[0].to(torch.float32)
            for r in range(1, world):  # same fixed rank order as the kernel
                v = vals[r].to(torch.float32)
                ref = ref + v if op == "sum" else (torch.maximum(ref, v) if op == "max" else torch.minimum(ref, v))
            errs.append(float((t.cpu() - ref).abs().max()))
            if it % 10 == 9:
                comm.barrier()
        comm.check()
        out["max_err"] = max(errs)
        # every rank must see bitwise-identical results
        t = torch.full((7,), 0.1 * (rank + 1), device=dev)
        comm.all_reduce_(t, "sum")
        allv: list = [None] * world
        dist.all_gather_object(allv, t.cpu().tolist())
        out["identical"] = all(v == allv[0] for v in allv)
        # timeout path: rank 0 calls alone with a short limit -> NaN + error
        dist.barrier()
        if rank == 0:
            comm._c.set_timeout(0.5)
            t = torch.ones(4, device=dev)
            comm.all_reduce_(t, "sum")
            torch.cuda.synchronize()
            out["timeout_nan"] = bool(torch.isnan(t).all())
            out["timeout_err"] = int(comm._c.error())
        dist.barrier()
        comm.close()
    except Exception as e:  # noqa: BLE001
        out["exc"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


@pytest.mark.gpu
def test_xgmi_allreduce_two_procs_one_gpu(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_xgmi_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        o = q.get(timeout=240)
        res[o["rank"]] = o
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert "exc" not in res[r], res[r]
        assert res[r]["created"], res[r]
        assert res[r]["max_err"] == 0.0, res[r]
        assert res[r]["identical"], res[r]
    assert res[0]["timeout_nan"] and res[0]["timeout_err"] == 1, res[0]


@pytest.mark.gpu
def test_xgmi_world1_and_roctx(gpu):
    from mxllm.parallel.xgmi import XgmiComm
    from mxllm.utils import profiling

    c = XgmiComm(0, 1, gpu, max_elems=256, timeout_s=5.0)
    c.open([c.handle()])
    assert c.self_test()
    t = torch.randn(200, device=gpu)
    ref = t.clone()
    c.all_reduce_(t, "sum")
    torch.testing.assert_close(t, ref, rtol=0, atol=0)
    c.close()
    assert torch.ops.mxllm.roctx_available()
    with profiling.range_("test-range"):
        profiling.mark("inside")


def _xgmi_graph_worker(rank, world, port, q):
    """Graph-safe bf16 all-reduce: eager calls of several sizes (multi-workgroup
    chunks), then the same calls captured once into a hipGraph and replayed
    with fresh inputs — exact vs the rank-ordered f32 sum, identical on ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_XGMI="1")
    import torch.distributed as dist

    from mxllm.parallel import xgmi

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"rank": rank}

    def vals(n, seed):
        return [torch.randn(n, generator=torch.Generator().manual_seed(seed * 31 + r)).to(torch.bfloat16)
                for r in range(world)]

    def want(vs):
        acc = vs[0].float()
        for v in vs[1:]:
            acc = acc + v.float()
        return acc.to(torch.bfloat16)

    try:
        comm = xgmi.create(dev, cls=xgmi.XgmiGraphComm, max_elems=1 << 17, timeout_s=30.0)
        out["created"] = comm is not None
        if comm is None:
            return
        ok = True
        for it, n in enumerate([8, 8192, 8200, 65536, 131072]):
            vs = vals(n, it)
            t = vs[rank].to(dev)
            comm.all_reduce_(t)
            ok &= bool(torch.equal(t.cpu(), want(vs)))
        out["eager_ok"] = ok
        # capture two reductions (decode-sized) into one graph, replay with new data
        a = torch.zeros(8192, dtype=torch.bfloat16, device=dev)
        b = torch.zeros(4 * 8192, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            comm.all_reduce_(a)
            comm.all_reduce_(b)
        ok = True
        for it in range(5):
            va, vb = vals(a.numel(), 100 + it), vals(b.numel(), 200 + it)
            a.copy_(va[rank])
            b.copy_(vb[rank])
            g.replay()
            torch.cuda.synchronize()
            ok &= bool(torch.equal(a.cpu(), want(va))) and bool(torch.equal(b.cpu(), want(vb)))
        comm.check()
        out["graph_ok"] = ok
        dist.barrier()
        comm.close()
    except Exception as e:  # noqa: BLE001
        out["exc"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


@pytest.mark.gpu
def test_xgmi_graph_allreduce_bf16_two_procs_one_gpu(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_xgmi_graph_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        o = q.get(timeout=240)
        res[o["rank"]] = o
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert "exc" not in res[r], res[r]
        assert res[r]["created"] and res[r]["eager_ok"] and res[r]["graph_ok"], res[r]
