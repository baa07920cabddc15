#!/usr/bin/env python3
"""gemm8 MFMA GEMM (4- and 8-phase schedules) (csrc/kernels/gemm8.hip) vs hipBLASLt on the Llama-3.1 training shapes.

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

from mxllm.ops import gemm, native  # noqa: E402
from mxllm.ops.linear import transpose2d  # noqa: E402

SHAPES = {
    # name: (out, in) of the projection weight
    "70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672),
            "head": (128256, 8192)},
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


# the path each form takes without gemm8 (what a table entry must beat)
DEFAULT = {"nn": "hipblaslt_nn", "tt": "transpose_tn", "tn": "hipblaslt_tn"}


def _ph4(fn):
    """the same call on the 4-phase schedule (MXLLM_GEMM8_PH=4, read per launch)"""
    def f():
        os.environ["MXLLM_GEMM8_PH"] = "4"
        try:
            fn()
        finally:
            os.environ.pop("MXLLM_GEMM8_PH", None)
    return f


def _persist(fn):
    """the same call on the persistent 4-phase kernel (MXLLM_GEMM8_PERSIST=1, read per launch)"""
    def f():
        os.environ["MXLLM_GEMM8_PH"] = "4"
        os.environ["MXLLM_GEMM8_PERSIST"] = "1"
        try:
            fn()
        finally:
            os.environ.pop("MXLLM_GEMM8_PH", None)
            os.environ.pop("MXLLM_GEMM8_PERSIST", None)
    return f


def run_case(name, flops, variants, rounds, calls):
    if os.environ.get("_G8_PH4_ALL") == "1" and "gemm8" in variants and "gemm8_ph4" not in variants:
        variants = dict(variants, gemm8_ph4=_ph4(variants["gemm8"]))
    if os.environ.get("_G8_PERSIST_ALL") == "1" and "gemm8" in variants and "gemm8_p" not in variants:
        variants = dict(variants, gemm8_p=_persist(variants["gemm8"]))
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
    ap.add_argument("--shapes", default="", help="comma list of projection names to run (default all)")
    ap.add_argument("--aug-only", action="store_true", help="only the --aug shapes")
    ap.add_argument("--aug", action="store_true",
                    help="also the 70B LoRA headline's augmented shapes (K + 64 pad, padded weight buffers) and head")
    ap.add_argument("--write-table", default=None,
                    help="write the shapes where gemm8 beats the default path by >= --margin (JSON for mxllm/ops/gemm.py)")
    ap.add_argument("--margin", type=float, default=0.01)
    ap.add_argument("--layout-exp", action="store_true", help="K-parity / row-stride experiment on the o dX shape")
    ap.add_argument("--layout-exp-only", action="store_true")
    ap.add_argument("--ablate", action="store_true", help="timing-only ablation builds of the NN kernel")
    ap.add_argument("--ph4", action="store_true", help="also time every gemm8 call on the 4-phase schedule")
    ap.add_argument("--persist", action="store_true", help="also time every gemm8 call on the persistent kernel")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if not a.no_table:
        from mxllm.utils import gemm_tuning

        print(json.dumps({"tuned_table": gemm_tuning.enable()}), flush=True)
    ops = native()
    T = a.tokens
    # warm the device (clocks, allocator, code objects) before the first timed case: in passes C
    # and D whichever case ran first read ~15 % slow (archive/profiles/r4d/layout.txt)
    wa, wb = rnd(4096, 8192, dev=dev), rnd(8192, 8192, dev=dev)
    wo = torch.empty(4096, 8192, device=dev, dtype=torch.bfloat16)
    import time as _t
    t_end = _t.time() + 3.0
    while _t.time() < t_end:
        for _ in range(20):
            ops.gemm8(wa, True, wb, False, wo, 0.0, None, 1.0)
            torch.mm(wa, wb, out=wo)
        torch.cuda.synchronize()
    del wa, wb, wo
    if a.ph4:
        os.environ["_G8_PH4_ALL"] = "1"
    if a.persist:
        os.environ["_G8_PERSIST_ALL"] = "1"
    forms = a.forms.split(",")
    models = [] if a.aug_only else (["70b", "8b"] if a.model == "both" else [a.model])
    a.aug = a.aug or a.aug_only
    only = set(filter(None, a.shapes.split(",")))
    results = []
    wins = []
    measured = set()

    def record(res, form, M, N, K, out):
        results.append(res)
        measured.add((form, M, N, K, out))
        ph, g, tail = 8, res["gemm8"]["ms"], 0
        if "gemm8_ph4" in res and res["gemm8_ph4"]["ms"] < g:
            ph, g = 4, res["gemm8_ph4"]["ms"]
        if "gemm8_p" in res and res["gemm8_p"]["ms"] < g:
            ph, g = 5, res["gemm8_p"]["ms"]  # ph 5 = the persistent 4-phase kernel (csrc/kernels/gemm8.hip)
        if "gemm8_tail" in res and res["gemm8_tail"]["ms"] < g:
            ph, g, tail = 4, res["gemm8_tail"]["ms"], gemm.tail_split(M, N, K)
        d = res[DEFAULT[form]]["ms"]
        if g < d * (1 - a.margin):
            e = {"form": form, "M": M, "N": N, "K": K, "out": out, "ph": ph,
                 "gemm8_tflops": round(2.0 * M * N * K / (g * 1e-3) / 1e12, 1),
                 "default_tflops": res[DEFAULT[form]]["tflops"], "case": res["case"]}
            if tail:
                e["tail"] = tail
            wins.append(e)

    def tail_variant(var, x, w, o, M, N, K, a_kc=True, b_kc=True):
        """the tail-balanced launch (mx_gemm8_tail) where the tile grid leaves a short last wave"""
        t = gemm.tail_split(M, N, K)
        if t:
            var["gemm8_tail"] = lambda: ops.gemm8_tail(x, a_kc, w, b_kc, o, abs(t), t < 0, 4)
        return var

    if a.ablate:
        # timing-only ablations of the NN kernel (results wrong): doubled MFMA per phase, no barriers
        M, N, K = T, 8192, 8192
        xa, wb = rnd(M, K, dev=dev), rnd(K, N, dev=dev)
        o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def var(v):
            def f():
                os.environ["MXLLM_GEMM8_ABLATE"] = str(v)
                ops.gemm8(xa, True, wb, False, o, 0.0, None, 1.0)
            return f
        def ph4():
            os.environ.pop("MXLLM_GEMM8_ABLATE", None)
            os.environ["MXLLM_GEMM8_PH"] = "4"
            ops.gemm8(xa, True, wb, False, o, 0.0, None, 1.0)
            os.environ.pop("MXLLM_GEMM8_PH", None)
        vs = {f"v{v}": var(v) for v in range(4)}
        vs["ph4"] = ph4
        res = run_case("ablate o dX nn (v0 real, v1 2x MFMA, v2 no barriers, v3 both; ph4 = 4-phase schedule)",
                       2.0 * M * N * K, vs, a.rounds, a.calls)
        os.environ.pop("MXLLM_GEMM8_ABLATE", None)
        results.append(res)
        if a.layout_exp_only:
            return
    if a.layout_exp:
        # why the 70B LoRA o-projection dX (K = 8192 + 64, padded buffers) runs ~17 % slower than the
        # plain shape in BOTH kernels: K-tile parity vs row stride of the operands
        for K, lda, ldb in ((8192, 8192, 8192), (8256, 8256, 8256), (8192, 8256, 8256), (8256, 8256, 8192),
                            (8256, 8320, 8320), (8320, 8320, 8320), (8192, 8320, 8320)):
            M, N = T, 8192
            xa = rnd(M, lda, dev=dev)[:, :K]
            wb = rnd(K, ldb, dev=dev)[:, :N]
            o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            record(run_case(f"layout o dX nn K{K} lda{lda} ldb{ldb}", 2.0 * M * N * K, {
                "gemm8": lambda: ops.gemm8(xa, True, wb, False, o, 0.0, None, 1.0),
                "hipblaslt_nn": lambda: torch.mm(xa, wb, out=o)}, a.rounds, a.calls), "nn", M, N, K, "bf16")
            del xa, wb, o
            torch.cuda.empty_cache()
        if a.layout_exp_only:
            return
    if a.aug:
        P = 64  # LoRA pad of every 70B projection (n * r rounded up to 64)
        for name, form, M, N, K, ldb in (("o dX", "nn", T, 8192, 8192 + P, 8192 + P),
                                         ("gu dX", "nn", T, 8192, 57344 + P, 8192 + P),
                                         ("down fwd (transposed buffer)", "nn", T, 8192, 28672 + P, 8192 + P),
                                         ("down fwd", "tn", T, 8192, 28672 + P, 28672 + P),
                                         ("head dX", "nn", T, 8192, 128256, 8192),
                                         ("qkv fwd", "tn", T, 10240, 8192 + P, 8192 + P),
                                         ("o fwd", "tn", T, 8192, 8192 + P, 8192 + P),
                                         ("gu fwd", "tn", T, 57344, 8192 + P, 8192 + P),
                                         ("qkv dX (image)", "tn", T, 8192, 10240 + P, 10240 + P),
                                         ("down dX (transposed buffer)", "tn", T, 28672, 8192 + P, 8192 + P),
                                         ("head fwd", "tn", T, 128256, 8192, 8192)):
            xa = rnd(M, K, dev=dev)
            o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            if form == "nn":
                wb = rnd(K, ldb, dev=dev)[:, :N]
                var = {"gemm8": lambda: ops.gemm8(xa, True, wb, False, o, 0.0, None, 1.0),
                       "hipblaslt_nn": lambda: torch.mm(xa, wb, out=o)}
            else:
                wb = rnd(N, K, dev=dev)
                var = tail_variant({"gemm8": lambda: ops.gemm8(xa, True, wb, True, o, 0.0, None, 1.0),
                                    "hipblaslt_tn": lambda: torch.mm(xa, wb.t(), out=o)}, xa, wb, o, M, N, K)
            if a.ph4:
                var["gemm8_ph4"] = _ph4(var["gemm8"])
            record(run_case(f"70b-lora {name} {form} M{M} N{N} K{K}", 2.0 * M * N * K, var, a.rounds, a.calls),
                   form, M, N, K, "bf16")
            del xa, wb, o
            torch.cuda.empty_cache()
    for mdl in models:
        for pname, (O, I) in SHAPES[mdl].items():
            if only and pname not in only:
                continue
            fl = 2.0 * T * O * I
            w = rnd(O, I, dev=dev)
            dy = rnd(T, O, dev=dev)
            x = rnd(T, I, dev=dev)
            if "nn" in forms and T % 256 == 0 and I % 256 == 0:
                o = torch.empty(T, I, device=dev, dtype=torch.bfloat16)
                record(run_case(f"{mdl} {pname} dX nn T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(dy, True, w, False, o, 0.0, None, 1.0),
                    "hipblaslt_nn": lambda: torch.mm(dy, w, out=o),
                }, a.rounds, a.calls), "nn", T, I, O, "bf16")
            if "tt" in forms and O % 256 == 0 and I % 256 == 0:
                o = torch.empty(O, I, device=dev, dtype=torch.bfloat16)
                record(run_case(f"{mdl} {pname} dW tt bf16 T{T}", fl, tail_variant({
                    "gemm8": lambda: ops.gemm8(dy, False, x, False, o, 0.0, None, 1.0),
                    "transpose_tn": lambda: torch.mm(transpose2d(dy), transpose2d(x).t(), out=o),
                    "hipblaslt_nt": lambda: torch.mm(dy.t(), x, out=o),
                }, dy, x, o, O, I, T, False, False), a.rounds, a.calls), "tt", O, I, T, "bf16")
            if "tt32" in forms and O % 256 == 0 and I % 256 == 0:
                o32 = torch.zeros(O, I, device=dev, dtype=torch.float32)
                record(run_case(f"{mdl} {pname} dW tt fp32+=  T{T}", fl, {
                    "gemm8": lambda: ops.gemm8(dy, False, x, False, o32, 1.0, None, 1.0),
                    "transpose_tn": lambda: torch.ops.aten.addmm.dtype_out(
                        o32, transpose2d(dy), transpose2d(x).t(), torch.float32, beta=1.0, out=o32),
                    "hipblaslt_nt": lambda: torch.ops.aten.addmm.dtype_out(o32, dy.t(), x, torch.float32, beta=1.0,
                                                                            out=o32),
                }, a.rounds, a.calls), "tt", O, I, T, "f32")
            if "tn" in forms and O % 256 == 0:
                o = torch.empty(T, O, device=dev, dtype=torch.bfloat16)
                record(run_case(f"{mdl} {pname} fwd tn T{T}", fl, tail_variant({
                    "gemm8": lambda: ops.gemm8(x, True, w, True, o, 0.0, None, 1.0),
                    "hipblaslt_tn": lambda: torch.mm(x, w.t(), out=o),
                }, x, w, o, T, O, I), a.rounds, a.calls), "tn", T, O, I, "bf16")
            del w, dy, x
            torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(results, f, indent=1)
    if a.write_table:
        old = []
        if os.path.exists(a.write_table):
            with open(a.write_table) as f:
                old = json.load(f).get("wins", [])
        key = lambda e: (e["form"], e["M"], e["N"], e["K"], e["out"])  # noqa: E731
        # entries of shapes not measured in this run are kept; measured shapes take this run's verdict
        merged = {key(e): e for e in old if key(e) not in measured}
        merged.update({key(e): e for e in wins})
        with open(a.write_table, "w") as f:
            json.dump({"arch": "gfx950", "source": "bench/gemm8_probe.py", "tokens": T, "margin": a.margin,
                       "wins": sorted(merged.values(), key=key)}, f, indent=1)
        print(json.dumps({"table": a.write_table, "wins": len(merged)}), flush=True)


if __name__ == "__main__":
    main()
