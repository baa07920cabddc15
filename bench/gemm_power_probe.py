#!/usr/bin/env python3
"""Clock and power of the GEMM kernels under sustained load (is the headline's GEMM time set by
instruction issue, or by the power cap?).

For one Llama-3.1-70B projection shape each variant runs back to back for ``--seconds``: hipBLASLt
TN (the tuned solution the headline uses), gemm8 TN / NN on the 4-phase schedule, and the
persistent gemm8.  Half-way through, one AMD SMI sample (mxllm/utils/gpumon.py) reads the graphics
clock and the socket power.  Reported per variant: TF/s, MHz, W, and TF/s per 1000 MHz (the
clock-normalised issue rate).  Variants alternate over ``--rounds``.
Usage: python bench/gemm_power_probe.py [--shape o|gu|down] [--tokens 4096] [--seconds 3] [--rounds 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mxllm.ops import native  # noqa: E402
from mxllm.utils.gpumon import sample_device  # noqa: E402

SHAPES = {"o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672), "qkv": (10240, 8192)}


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def run(name, fn, flops, seconds):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    per = time.perf_counter() - t0
    n = max(10, int(seconds / max(per, 1e-4)))
    sample = {}

    def probe():
        time.sleep(seconds / 2)
        sample.update(sample_device(0))

    th = threading.Thread(target=probe)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    th.start()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    th.join()
    ms = a.elapsed_time(b) / n
    tf = flops / ms / 1e9
    mhz = sample.get("gfx_clock_mhz")
    return {"variant": name, "ms": round(ms, 4), "tflops": round(tf, 1), "gfx_clock_mhz": mhz,
            "socket_power_w": sample.get("socket_power_w"),
            "tflops_per_ghz": round(tf / (mhz / 1000.0), 1) if mhz else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="o", choices=sorted(SHAPES))
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    ops = native()
    N, K = SHAPES[a.shape]
    M = a.tokens
    x = rnd(M, K)
    w = rnd(N, K)
    wt = w.t().contiguous()  # [K, N] n-contiguous: the NN form of the same product
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    flops = 2.0 * M * N * K
    variants = {
        "hipblaslt_tn": lambda: torch.mm(x, w.t(), out=out),
        "gemm8_tn_ph4": lambda: ops.gemm8(x, True, w, True, out, 0.0, None, 1.0, 4),
        "gemm8_nn_ph4": lambda: ops.gemm8(x, True, wt, False, out, 0.0, None, 1.0, 4),
        "gemm8_tn_persistent": lambda: ops.gemm8(x, True, w, True, out, 0.0, None, 1.0, 5),
    }
    for r in range(a.rounds):
        for name, fn in variants.items():
            res = run(name, fn, flops, a.seconds)
            res.update(shape=f"70b {a.shape} M{M} N{N} K{K}", round=r)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
