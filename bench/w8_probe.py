#!/usr/bin/env python3
"""fp8-weight decode GEMM (csrc/kernels/fp8_gemm.hip w8a16_gemm_kernel) at the Llama-3.1-70B / 8B
projection shapes: achieved weight-streaming bandwidth per channel-group count (MXLLM_W8_NC, read
per call), variants interleaved in one process (median of per-call events, median over rounds).
Usage: python bench/w8_probe.py [--ms 1,4,8] [--nc 0,1,2,4] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mxllm.ops import native  # noqa: E402
from mxllm.serve.quant import quantize_e4m3  # noqa: E402

SHAPES = {"70b qkv": (8192, 10240), "70b o": (8192, 8192), "70b gu": (8192, 57344), "70b down": (28672, 8192),
          "8b qkv": (4096, 6144), "8b gu": (4096, 28672), "8b down": (14336, 4096)}


def time_us(fn, calls):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return 1e3 * statistics.median(s.elapsed_time(e) for s, e in ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,4,8")
    ap.add_argument("--nc", default="0,1,2,4", help="0 = the default rule")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = native()
    out = []
    for name, (K, N) in SHAPES.items():
        q, sc = quantize_e4m3((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
        for M in map(int, a.ms.split(",")):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            res = {nc: [] for nc in a.nc.split(",")}
            ref = None
            for _ in range(a.rounds):
                for nc in res:
                    os.environ["MXLLM_W8_NC"] = nc if nc != "0" else ""
                    y = ops.w8_linear(x, q, sc)
                    if ref is None:
                        ref = y.float()
                    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3, (name, M, nc)
                    res[nc].append(time_us(lambda: ops.w8_linear(x, q, sc), a.calls))
            os.environ.pop("MXLLM_W8_NC", None)
            rec = {"case": f"{name} M{M} N{N} K{K}", "weight_mb": round(N * K / 1e6, 1)}
            for nc, v in res.items():
                us = statistics.median(v)
                rec[f"nc{nc}"] = {"us": round(us, 1), "tbps": round(N * K / (us * 1e-6) / 1e12, 2)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        del q, sc
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
