#!/usr/bin/env python3
"""Fused forward epilogues (csrc/kernels/gemm8.hip G8_EPI_ROPE / G8_EPI_SWIGLU) in isolation, at
the Llama-3.1 8B / 70B training shapes (T tokens): the fused GEMM vs the same gemm8 GEMM followed
by the kernel it replaces (rope_split / swiglu_fwd) vs hipBLASLt + that kernel.  Interleaved
rounds in one process, median of back-to-back calls; prints one JSON line per case (ms, TF/s of
the GEMM).  Usage: python bench/fused_epi_bench.py [--tokens 4096] [--rounds 5]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.ops import native  # noqa: E402
from mxllm.ops import reference as ref  # noqa: E402


def time_ms(fn, calls=5):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) for s, e in ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = native()
    T = a.tokens
    S = 2048
    B = T // S
    cos, sin = ref.rope_tables(S, 128, 500000.0, {"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                  "original_max_position_embeddings": 8192}, dev)

    def rnd(*shape):
        return (torch.rand(*shape, device=dev) * 2 - 1).to(torch.bfloat16)

    for name, H, Hq, Hkv, F in (("8b", 4096, 32, 8, 14336), ("70b", 8192, 64, 8, 28672)):
        x = rnd(T, H)
        # qkv + RoPE
        N = (Hq + 2 * Hkv) * 128
        w = rnd(N, H) * 0.05
        q = torch.empty(B, Hq, S, 128, device=dev, dtype=torch.bfloat16)
        k = torch.empty(B, Hkv, S, 128, device=dev, dtype=torch.bfloat16)
        v = torch.empty_like(k)
        qkv = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        var = {
            "fused_gemm8": lambda: ops.gemm8_rope(x, w, cos, sin, B, S, Hq, Hkv, q, k, v),
            "gemm8_only": lambda: ops.gemm8(x, True, w, True, qkv, 0.0, None, 1.0, 4),
            "gemm8+rope_split": lambda: (ops.gemm8(x, True, w, True, qkv, 0.0, None, 1.0, 4),
                                         ops.rope_split(qkv, cos, sin, B, S, Hq, Hkv, 128)),
            "hipblaslt_only": lambda: torch.mm(x, w.t(), out=qkv),
            "hipblaslt+rope_split": lambda: (torch.mm(x, w.t(), out=qkv), ops.rope_split(qkv, cos, sin, B, S, Hq, Hkv, 128)),
        }
        report(f"{name} qkv+rope T{T}", 2 * T * H * N, var, a.rounds)
        # gate-up + SwiGLU
        w2 = rnd(2 * F, H) * 0.05
        gu = torch.empty(T, 2 * F, device=dev, dtype=torch.bfloat16)
        m = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
        var = {
            "fused_gemm8": lambda: ops.gemm8_swiglu(x, w2, gu, m),
            "gemm8_only": lambda: ops.gemm8(x, True, w2, True, gu, 0.0, None, 1.0, 4),
            "gemm8+swiglu": lambda: (ops.gemm8(x, True, w2, True, gu, 0.0, None, 1.0, 4), ops.swiglu_fwd(gu, 0)),
            "hipblaslt_only": lambda: torch.mm(x, w2.t(), out=gu),
            "hipblaslt+swiglu": lambda: (torch.mm(x, w2.t(), out=gu), ops.swiglu_fwd(gu, 0)),
        }
        report(f"{name} gu+swiglu T{T}", 2 * T * H * 2 * F, var, a.rounds)


def report(case, flops, var, rounds):
    res = {k: [] for k in var}
    for _ in range(rounds):
        for k, fn in var.items():
            res[k].append(time_ms(fn))
    out = {"case": case}
    for k, v in res.items():
        ms = statistics.median(v)
        out[k] = {"ms": round(ms, 4), "gemm_tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
