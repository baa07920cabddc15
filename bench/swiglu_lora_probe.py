#!/usr/bin/env python3
"""SwiGLU fused with the LoRA tail (csrc/kernels/lora.hip swiglu_lora_kernel) vs the unfused pair
(swiglu kernel + lora_xwt re-reading its output), at the Llama-3.1 70B / 8B LoRA shapes.

Variants run interleaved in one process (R rounds, median of `calls` per round); `--cs` sweeps the
column-split count (MXLLM_SWIGLU_LORA_CS, read per launch).
Usage: python bench/swiglu_lora_probe.py [--tokens 4096] [--rounds 5] [--cs 0,4,8,16]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--cs", default="0")
    ap.add_argument("--rbw", default="1", help="16-row blocks per workgroup (MXLLM_SWIGLU_LORA_RBW)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = native()
    T, pad, s = a.tokens, 64, 2.0
    out = []
    for name, F, r_d, r_gu in (("70b", 28672, 16, 32), ("8b", 14336, 16, 32)):
        gu = torch.randn(T, 2 * F, device=dev, dtype=torch.bfloat16)
        dm = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
        a_d = torch.zeros(pad, F + pad, device=dev, dtype=torch.bfloat16)[:, :F]  # A rows in wbuf [pad, K+pad]
        a_d[:r_d] = torch.randn(r_d, F, device=dev, dtype=torch.bfloat16) * 0.01
        bt_gu = torch.zeros(pad, 2 * F, device=dev, dtype=torch.bfloat16)  # wbt [pad, N]
        bt_gu[:r_gu] = torch.randn(r_gu, 2 * F, device=dev, dtype=torch.bfloat16) * 0.01
        for direction in ("fwd", "bwd"):
            if direction == "fwd":
                def unfused():
                    m = ops.swiglu_fwd(gu, pad)
                    full = m.as_strided((T, F + pad), (F + pad, 1))
                    ops.lora_xwt(m, a_d, full[:, F:], s)

                def plain():
                    ops.swiglu_fwd(gu, pad)
                fused = {f"fused_r{rb}_cs{c}": (lambda c=c, rb=rb: (os.environ.__setitem__("MXLLM_SWIGLU_LORA_CS", str(c)),
                                                                   os.environ.__setitem__("MXLLM_SWIGLU_LORA_RBW", rb),
                                                                   ops.swiglu_lora(None, gu, pad, a_d, r_d // 16, s)))
                         for c in map(int, a.cs.split(",")) for rb in a.rbw.split(",")}
                nbytes = 3 * T * F * 2
            else:
                def unfused():
                    d = ops.swiglu_bwd(dm, gu, pad)
                    full = d.as_strided((T, 2 * F + pad), (2 * F + pad, 1))
                    ops.lora_xwt(d, bt_gu, full[:, 2 * F:], s)

                def plain():
                    ops.swiglu_bwd(dm, gu, pad)
                fused = {f"fused_r{rb}_cs{c}": (lambda c=c, rb=rb: (os.environ.__setitem__("MXLLM_SWIGLU_LORA_CS", str(c)),
                                                                   os.environ.__setitem__("MXLLM_SWIGLU_LORA_RBW", rb),
                                                                   ops.swiglu_lora(dm, gu, pad, bt_gu, r_gu // 16, s)))
                         for c in map(int, a.cs.split(",")) for rb in a.rbw.split(",")}
                nbytes = 5 * T * F * 2
            variants = {"unfused": unfused, "swiglu_only": plain, **fused}
            res = {k: [] for k in variants}
            for _ in range(a.rounds):
                for k, fn in variants.items():
                    res[k].append(time_us(fn, a.calls))
            rec = {"case": f"{name} {direction} T{T} F{F}", "swiglu_bytes_gb": round(nbytes / 1e9, 3)}
            for k, v in res.items():
                us = statistics.median(v)
                rec[k] = {"us": round(us, 1), "swiglu_tbps": round(nbytes / (us * 1e-6) / 1e12, 2)}
            os.environ.pop("MXLLM_SWIGLU_LORA_CS", None)
            os.environ.pop("MXLLM_SWIGLU_LORA_RBW", None)
            print(json.dumps(rec), flush=True)
            out.append(rec)
        del gu, dm, a_d, bt_gu
        torch.cuda.empty_cache()
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
