#!/usr/bin/env python3
"""How much a bulk collective running beside a GEMM costs the GEMM (VERDICT r4 Weak 7: "nothing in the
repo measures contention between collective kernels and gemm8 on one GPU").

Two processes share the box's one MI355X; their reduce-scatters run through the peer-memory
collectives (``MXLLM_COMM=peer``, csrc/kernels/peer_coll.hip: the same kernel a rank runs against its
7 peers over xGMI, here against one peer through HBM) on each communicator's own stream, exactly as
the ZeRO-3 trainer issues them.  Rank 0 also runs a stream of gemm8 GEMMs (the 70B config-4 dX shape,
T 8192 x 8192 x K 8192, NN) on its compute stream.  Three phases:
  A  GEMMs alone                      -> ms per GEMM
  B  reduce-scatters alone            -> GB/s of reduce-scatter input per rank
  C  both at once (the collectives enqueued first, then the GEMMs) -> GEMM slowdown, collective rate
Both ranks' collective kernels land on the one GPU, so phase C charges the GEMM with TWO ranks' worth
of collective workgroups: an upper bound on what one rank's collectives cost its GPU at world 8.
Usage: python bench/comm_contention_probe.py [--mb 256] [--reps 20] [--gemms 40]
       [--configs resident:32,light:64,light:128,light:128:bf16]
Prints one JSON line per configuration (schedule, workgroups, wire dtype).  GB/s counts fp32
reduce-scatter input per rank (a bf16 wire moves half those bytes).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, a, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MXLLM_BACKEND="gloo", MXLLM_COMM="peer",
                      MXLLM_COMM_STRICT="1", MXLLM_PEER_WGS=str(min(a.wgs, 64) if a.algo == "resident" else 8),
                      MXLLM_PEER_TIMEOUT_S="120", MXLLM_PEER_ALGO=a.algo, MXLLM_PEER_LIGHT_WGS=str(a.wgs),
                      MXLLM_PEER_LIGHT_MB=str(a.light_mb))
    import torch.distributed as dist

    from mxllm.ops import native
    from mxllm.parallel import runtime
    from mxllm.parallel.comm import create

    env = runtime.init(rank=rank, world_size=world)
    dev = env.device
    comm = create(None, dev)
    m = a.mb * (1 << 20) // 4 // world  # fp32 elements of each rank's output chunk
    x = torch.randn(world * m, device=dev)
    out = torch.empty(m, device=dev)
    ops = native()
    T, N, K = 8192, 8192, 8192
    ga = (torch.rand(T, K, device=dev) - 0.5).to(torch.bfloat16)
    gb = (torch.rand(K, N, device=dev) - 0.5).to(torch.bfloat16)
    gc = torch.empty(T, N, device=dev, dtype=torch.bfloat16)

    def gemms(n: int) -> float:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            assert ops.gemm8(ga, True, gb, False, gc, 0.0, None, 1.0, 4)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    wire = torch.bfloat16 if a.wire == "bf16" else None

    def colls(n: int):
        works = [comm.reduce_scatter(out, x, async_op=True, wire=wire) for _ in range(n)]
        return works

    res = {"rank": rank}
    if rank == 0:
        gemms(5)  # warm
    for w in colls(3):
        w.wait()
    torch.cuda.synchronize()
    dist.barrier()
    # A: GEMMs alone
    if rank == 0:
        res["gemm_ms_alone"] = gemms(a.gemms)
    dist.barrier()
    # B: reduce-scatters alone
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for w in colls(a.reps):
        w.wait()
    torch.cuda.synchronize()
    tb = time.perf_counter() - t0
    dist.barrier()
    res["rs_gbs_alone"] = a.reps * world * m * 4 / tb / 1e9
    # C: both, with as many reduce-scatters as cover the GEMM stream (so every GEMM runs beside them)
    n_c = [0]
    if rank == 0:
        n_c[0] = max(2, round(res["gemm_ms_alone"] * a.gemms / (1e3 * tb / a.reps)))
    dist.broadcast_object_list(n_c, src=0)
    res["rs_calls_beside_gemm"] = n_c[0]
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    works = colls(n_c[0])
    if rank == 0:
        res["gemm_ms_with_rs"] = gemms(a.gemms)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    tc = time.perf_counter() - t0
    dist.barrier()
    res["rs_gbs_with_gemm"] = n_c[0] * world * m * 4 / tc / 1e9
    runtime.cleanup()
    q.put(res)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256, help="reduce-scatter input MB per rank per call")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--gemms", type=int, default=40)
    ap.add_argument("--light-mb", type=int, default=64, help="MXLLM_PEER_LIGHT_MB (slot size of the light schedule)")
    ap.add_argument("--configs", default="resident:32,light:64,light:128",
                    help="comma list of schedule:workgroups[:bf16] (MXLLM_PEER_ALGO, its workgroups, a bf16 wire)")
    a = ap.parse_args()
    world = 2
    for spec in a.configs.split(","):
        parts = spec.split(":")
        a.algo, wgs, a.wire = parts[0], int(parts[1]), (parts[2] if len(parts) > 2 else "fp32")
        a.wgs = wgs
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, a, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = {}
        for _ in range(world):
            o = q.get(timeout=600)
            res[o["rank"]] = o
        for p in ps:
            p.join(60)
        r0 = res[0]
        line = {"schedule": a.algo, "peer_wgs": wgs, "wire": a.wire, "rs_mb_per_call": a.mb,
                "rs_calls_beside_gemm": r0["rs_calls_beside_gemm"], "gemm": "gemm8 NN 8192x8192x8192",
                "gemm_ms_alone": round(r0["gemm_ms_alone"], 4), "gemm_ms_with_rs": round(r0["gemm_ms_with_rs"], 4),
                "gemm_slowdown_pct": round(100 * (r0["gemm_ms_with_rs"] / r0["gemm_ms_alone"] - 1), 2),
                "rs_gbs_alone": round(min(o["rs_gbs_alone"] for o in res.values()), 1),
                "rs_gbs_with_gemm": round(min(o["rs_gbs_with_gemm"] for o in res.values()), 1)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
