#!/usr/bin/env python3
"""Does a TunableOp table entry change a GEMM's time?  Times y = x W^T for one (N, M, K) shape with
the library default and then with ``--table`` loaded read-only (mxllm/utils/gemm_tuning.py), with
weights rotated through more than the 256 MB Infinity Cache, and prints the kernel each picks
(from the profiler).  Usage: python bench/tunable_check.py --table t.csv [--n 57344 --m 4096 --k 8256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(x, ws, iters=30):
    for w in ws[:2]:
        torch.mm(x, w.t())
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(iters):
        torch.mm(x, ws[i % len(ws)].t())
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def kernels(x, w):
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as p:
        torch.mm(x, w.t())
        torch.cuda.synchronize()
    return sorted({e.name[:90] for e in p.events() if e.device_type == torch.autograd.DeviceType.CUDA})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", required=True)
    ap.add_argument("--n", type=int, default=57344)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--k", type=int, default=8256)
    a = ap.parse_args()
    x = torch.randn(a.m, a.k, device="cuda", dtype=torch.bfloat16)
    copies = max(2, (600 << 20) // (a.n * a.k * 2) + 1)
    ws = [torch.randn(a.n, a.k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    flops = 2 * a.m * a.n * a.k
    t0 = run(x, ws)
    k0 = kernels(x, ws[0])
    from mxllm.utils import gemm_tuning

    os.environ["MXLLM_GEMM_TABLE"] = a.table
    on = gemm_tuning.enable(a.table)
    t1 = run(x, ws)
    k1 = kernels(x, ws[0])
    print(json.dumps({"shape": [a.m, a.n, a.k], "default_ms": round(t0, 4), "default_tf": round(flops / t0 / 1e9),
                      "default_kernels": k0, "table_on": on, "table_ms": round(t1, 4),
                      "table_tf": round(flops / t1 / 1e9), "table_kernels": k1}), flush=True)


if __name__ == "__main__":
    main()
