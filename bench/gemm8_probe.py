#!/usr/bin/env python3
"""8-phase MFMA GEMM (csrc/kernels/gemm8.hip) vs hipBLASLt on the Llama-3.1 training shapes.

For every shape the variants run interleaved in ONE process (guide §5.4 rule 24): R rounds, each
round times every variant (median of `--calls` back-to-back calls after warm-up); reported is the
median over rounds in TF/s, on uniform random [-1, 1) operands.

Forms (T = tokens):
  nn  dX = dY W            : gemm8(dY k-contig, W mn-contig)  vs  torch.mm(dY, W)      (hipBLASLt "NN")
  tt  dW = dY^T X          : gemm8(dY, X both token-major)    vs  transpose2d x2 + mm  (current default)
                                                               and torch.mm(dY.t(), X) (hipBLASLt "NT")
  tt32 same, fp32 output accumulated (beta 1)                   vs  the same two paths with fp32 out
  tn  y = x W^T            : gemm8(x, W both k-contig)         vs  torch.mm(x, W.t())   (reference point)
Usage: python bench/gemm8_probe.py [--model 70b|8b|both] [--rounds 5] [--json-out F]
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
from mxllm.ops.linear import transpose2d  # noqa: E402

SHAPES = {
    # name: (out, in) of the projection weight
    "70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672)},
    "8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336),
           "head": (128256, 4096)},
}


def rnd(*shape, dev):
    return (torch.rand(*shape, device=dev) * 2 - 1).to(torch.bfloat16)


def time_ms(fn, calls):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) for s, e in ev)


def run_case(name, flops, variants, rounds, calls):
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            res[k].append(time_ms(fn, calls))
    out = {"case": name}
    for k, v in res.items():
        ms = statistics.median(v)
        out[k] = {"ms": round(ms, 4), "tflops": round(flops / (ms * 1e-3) / 1e12, 1)}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="both")
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--forms", default="nn,tt,tt32,tn")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-table", action="store_true", help="hipBLASLt defaults instead of the tuned table")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if not a.no_table:
        from mxllm.utils import gemm_tuning

        print(json.dumps({"tuned_table": gemm_tuning.enable()}), flush=True)
    ops = native()
    T = a.tokens
    forms = a.forms.split(",")
    models = ["70b", "8b"] if a.model == "both" else [a.model]
    results = []
    for mdl in models:
        for pname, (O, I) in SHAPES[mdl].items():
            fl = 2.0 * T * O * I
            w = rnd(O, I, dev=dev)
            dy = rnd(T, O, dev=dev)
            x = rnd(T, I, dev=dev)
            if "nn" in forms and T % 256 == 0 and I % 256 == 0:
                o = torch.empty(T, I, device=dev, dtype=torch.bfloat16)
                results.append(run_case(f"{mdl} {pname} dX nn T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(dy, True, w, False, o, 0.0, None, 1.0),
                    "hipblaslt_nn": lambda: torch.mm(dy, w, out=o),
                }, a.rounds, a.calls))
            if "tt" in forms and O % 256 == 0 and I % 256 == 0:
                o = torch.empty(O, I, device=dev, dtype=torch.bfloat16)
                results.append(run_case(f"{mdl} {pname} dW tt bf16 T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(dy, False, x, False, o, 0.0, None, 1.0),
                    "transpose_tn": lambda: torch.mm(transpose2d(dy), transpose2d(x).t(), out=o),
                    "hipblaslt_nt": lambda: torch.mm(dy.t(), x, out=o),
                }, a.rounds, a.calls))
            if "tt32" in forms and O % 256 == 0 and I % 256 == 0:
                o32 = torch.zeros(O, I, device=dev, dtype=torch.float32)
                results.append(run_case(f"{mdl} {pname} dW tt fp32+=  T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(dy, False, x, False, o32, 1.0, None, 1.0),
                    "transpose_tn": lambda: torch.ops.aten.addmm.dtype_out(
                        o32, transpose2d(dy), transpose2d(x).t(), torch.float32, beta=1.0, out=o32),
                    "hipblaslt_nt": lambda: torch.ops.aten.addmm.dtype_out(o32, dy.t(), x, torch.float32, beta=1.0,
                                                                            out=o32),
                }, a.rounds, a.calls))
            if "tn" in forms and O % 256 == 0:
                o = torch.empty(T, O, device=dev, dtype=torch.bfloat16)
                results.append(run_case(f"{mdl} {pname} fwd tn T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(x, True, w, True, o, 0.0, None, 1.0),
                    "hipblaslt_tn": lambda: torch.mm(x, w.t(), out=o),
                }, a.rounds, a.calls))
            del w, dy, x
            torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
