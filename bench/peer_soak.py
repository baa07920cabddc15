#!/usr/bin/env python3
"""Soak test of the peer-memory collectives (light schedule by default): W processes share the box's
GPU and run thousands of back-to-back reduce-scatter / all-gather / all-reduce calls of random sizes
(several segments each with a small ``MXLLM_PEER_LIGHT_MB``), two communicators in flight at once,
fp32 / bf16 / the bf16 wire, every result checked bit for bit against the rank-ordered fp32 sum.
A protocol race (a slot overwritten before its consumer read it, a flag seen before its data) shows
up as a mismatch or a timeout.  Prints one JSON line per rank count.

Usage: python bench/peer_soak.py [--worlds 2,4] [--iters 400] [--algo light]
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
                      MXLLM_COMM_STRICT="1", MXLLM_PEER_ALGO=a.algo, MXLLM_PEER_LIGHT_MB=str(a.light_mb),
                      MXLLM_PEER_TIMEOUT_S="60", MXLLM_PEER_WGS="8")
    out = {"rank": rank}
    try:
        import torch.distributed as dist

        from mxllm.parallel import runtime
        from mxllm.parallel.comm import create

        env = runtime.init(rank=rank, world_size=world)
        dev = env.device
        c1, c2 = create(None, dev), create(dist.new_group(), dev)
        g = torch.Generator().manual_seed(1234)  # the same size / dtype sequence on every rank
        bad, calls, t0 = 0, 0, time.time()
        for it in range(a.iters):
            m = int(torch.randint(1, 1 << 17, (1,), generator=g)) * 8  # up to 1M elements per rank chunk
            kind = int(torch.randint(0, 3, (1,), generator=g))
            dt = torch.float32 if kind != 1 else torch.bfloat16
            wire = torch.bfloat16 if (kind == 2 and a.algo == "light") else None
            # deterministic per-(iteration, rank) data, small integers: every sum is exact in fp32
            base = torch.arange(world * m, device=dev, dtype=torch.float32)
            vals = [((base * 7 + it * 13 + r * 5) % 17 - 8) for r in range(world)]
            x = vals[rank].to(dt)
            rs = torch.empty(m, dtype=dt, device=dev)
            w1 = c1.reduce_scatter(rs, x, async_op=True, wire=wire) if wire is not None else \
                c1.reduce_scatter(rs, x, async_op=True)
            ag_in = ((torch.arange(m, device=dev, dtype=torch.float32) + it + rank) % 29).to(dt)
            ag = torch.empty(world * m, dtype=dt, device=dev)
            w2 = c2.all_gather(ag, ag_in, async_op=True)
            ar = vals[rank][: max(8, m * world - 8 * (it % 3))].to(dt).clone()  # sizes that need padding too
            c1.all_reduce(ar)
            w1.wait()
            w2.wait()
            want_rs = sum(v.to(dt).float() for v in vals).view(world, m)[rank].to(dt)
            want_ag = torch.cat([((torch.arange(m, device=dev, dtype=torch.float32) + it + r) % 29).to(dt)
                                 for r in range(world)])
            want_ar = sum(v[: ar.numel()].to(dt).float() for v in vals).to(dt)
            ok = (torch.equal(rs, want_rs) and torch.equal(ag, want_ag) and torch.equal(ar, want_ar))
            bad += 0 if ok else 1
            calls += 3
        torch.cuda.synchronize()
        c1.check()
        c2.check()
        out.update(calls=calls, mismatches=bad, seconds=round(time.time() - t0, 1))
        dist.barrier()
        runtime.cleanup()
    except Exception as e:  # noqa: BLE001
        out["error"] = f"{type(e).__name__}: {e}"[:500]
    q.put(out)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4")
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--algo", default="light")
    ap.add_argument("--light-mb", type=int, default=1, help="small slots: most calls run as several segments")
    a = ap.parse_args()
    for world in [int(w) for w in a.worlds.split(",")]:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, a, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = [q.get(timeout=1200) for _ in range(world)]
        for p in ps:
            p.join(60)
        line = {"algo": a.algo, "world": world, "iters": a.iters, "light_mb": a.light_mb,
                "calls_per_rank": max(r.get("calls", 0) for r in res),
                "mismatches": sum(r.get("mismatches", 0) for r in res),
                "errors": [r["error"] for r in res if "error" in r],
                "seconds": max(r.get("seconds", 0) for r in res)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
