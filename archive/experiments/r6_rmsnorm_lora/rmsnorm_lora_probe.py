#!/usr/bin/env python3
"""Time the fused RMSNorm + LoRA tail (rmsnorm_lora_fwd) against the rmsnorm_fwd + lora_xwt pair it
replaces, at the 70B-LoRA headline shapes (T 4096, H 8192; 48 adapter rows = q/k/v, 32 = gate-up).
Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    from mxllm.ops._ext import native

    ops = native()
    dev = torch.device("cuda", 0)
    T, pad, eps, alpha = 4096, 64, 1e-5, 2.0
    for H, rows in ((8192, 48), (8192, 32), (4096, 48)):
        x = torch.randn(T, H, device=dev).bfloat16()
        res = torch.randn(T, H, device=dev).bfloat16()
        w = torch.ones(H, device=dev, dtype=torch.bfloat16)
        vbuf = torch.zeros(64, H + pad, device=dev, dtype=torch.bfloat16)
        vbuf[:rows, :H] = (0.02 * torch.randn(rows, H, device=dev)).bfloat16()
        v = vbuf[:, :H]

        def unfused():
            y, _, _ = ops.rmsnorm_fwd(x, res, w, eps, pad)
            ops.lora_xwt(y, v, y.as_strided((T, H + pad), (H + pad, 1))[:, H:], alpha, rows)

        def norm_only():
            ops.rmsnorm_fwd(x, res, w, eps, pad)

        def fused():
            ops.rmsnorm_lora_fwd(x, res, w, eps, pad, v, alpha, rows)

        r = {"T": T, "H": H, "rows": rows, "unfused_us": round(timeit(unfused), 1),
             "norm_only_us": round(timeit(norm_only), 1), "fused_us": round(timeit(fused), 1)}
        for dbg in ("1", "2"):
            os.environ["MXLLM_NL_DBG"] = dbg
            r["fused_dbg" + dbg + "_us"] = round(timeit(fused), 1)
            del os.environ["MXLLM_NL_DBG"]
        r["fused_tb_s"] = round(4 * T * H * 2 / (r["fused_us"] * 1e-6) / 1e12, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
