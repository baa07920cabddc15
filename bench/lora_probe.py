#!/usr/bin/env python3
"""LoRA rank-r kernels (csrc/kernels/lora.hip) at the Llama-3.1-70B headline shapes: achieved HBM
bandwidth of ``lora_xwt`` (s x A^T / s dy B tails: the row-tiled kernel on the adapter rows vs the
64-row LDS-DMA kernel on all padded rows) and ``lora_grads`` (dA and every dB_i in one launch) per
projection, the latter for several workgroup targets (MXLLM_LORA_WGS, read per launch).

Both sweep the workgroup target (MXLLM_LORA_WGS, read per launch) over ``--wgs``.
Usage: python bench/lora_probe.py [--tokens 4096] [--wgs 256,512,1024] [--rounds 5]
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

# projection: (in K, splits of N), r = 16, pad 64 (70B)
PROJ = {"qkv": (8192, [8192, 1024, 1024]), "o": (8192, [8192]), "gu": (8192, [28672, 28672]),
        "down": (28672, [8192])}


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
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--wgs", default="256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = native()
    T, r, pad, s = a.tokens, 16, 64, 2.0
    wgs = [int(w) for w in a.wgs.split(",")]
    out = []
    for name, (K, splits) in PROJ.items():
        N, R = sum(splits), r * len(splits)
        xa = torch.randn(T, K + pad, device=dev, dtype=torch.bfloat16)
        dya = torch.randn(T, N + pad, device=dev, dtype=torch.bfloat16)
        A = torch.randn(pad, K, device=dev, dtype=torch.bfloat16) * 0.01
        Bt = torch.randn(pad, N, device=dev, dtype=torch.bfloat16) * 0.01
        ga = torch.empty(R, K, device=dev, dtype=torch.bfloat16)
        gb = torch.zeros(N, R, device=dev, dtype=torch.bfloat16)
        x, dy = xa[:, :K], dya[:, :N]
        def xwt(mode, X, V, tail):
            def f():
                if mode in ("lds", "lds_fused", "lds_red64"):
                    os.environ["MXLLM_LORA_XWT"] = "lds"
                    os.environ["MXLLM_LORA_FUSED_RED"] = "1" if mode == "lds_fused" else "0"
                    os.environ["MXLLM_LORA_XWT_RED_ROWS"] = "64" if mode == "lds_red64" else "16"
                    ops.lora_xwt(X, V, tail, s)
                else:
                    os.environ["MXLLM_LORA_XWT"] = "tile"
                    ops.lora_xwt(X, V, tail, s, R)
            return f

        for cname, X, V, tail, nbytes in (("xwt_x", x, A, xa[:, K:], T * K * 2), ("xwt_dy", dy, Bt, dya[:, N:], T * N * 2)):
            res = {f"lds_wgs{w}": [] for w in wgs}
            for _ in range(a.rounds):
                for m in res:
                    os.environ["MXLLM_LORA_WGS"] = m.split("wgs")[1]
                    res[m].append(time_us(xwt("lds", X, V, tail), a.calls))
            os.environ.pop("MXLLM_LORA_WGS", None)
            os.environ.pop("MXLLM_LORA_XWT", None)
            os.environ.pop("MXLLM_LORA_FUSED_RED", None)
            os.environ.pop("MXLLM_LORA_XWT_RED_ROWS", None)
            rec = {"case": f"70b {name} {cname} T{T} R{R}", "gb": round(nbytes / 1e9, 3)}
            for m, v in res.items():
                us = statistics.median(v)
                rec[m] = {"us": round(us, 1), "tbps": round(nbytes / (us * 1e-6) / 1e12, 2)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        fn, nbytes = (lambda: ops.lora_grads(x, dy, dya[:, N:], xa[:, K:], ga, gb, splits, r, True)), T * (K + N) * 2
        res = {w: [] for w in wgs}
        for _ in range(a.rounds):
            for w in res:
                os.environ["MXLLM_LORA_WGS"] = str(w)
                res[w].append(time_us(fn, a.calls))
        os.environ.pop("MXLLM_LORA_WGS", None)
        os.environ.pop("MXLLM_LORA_FUSED_RED", None)
        rec = {"case": f"70b {name} grads T{T}", "gb": round(nbytes / 1e9, 3)}
        for w, v in res.items():
            us = statistics.median(v)
            rec[f"wgs{w}"] = {"us": round(us, 1), "tbps": round(nbytes / (us * 1e-6) / 1e12, 2)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del xa, dya, A, Bt, ga, gb
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
