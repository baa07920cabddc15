"""Decode-GEMM microbenchmark: y = x W^T with 1..32 (hipBLASLt also 64) token rows at the Llama-3.1 8B / 70B
projection shapes, hipBLASLt (F.linear) vs the weight-streaming HIP kernel
(csrc/kernels/skinny_gemm.hip).  Weights are cycled through enough copies to exceed the
256 MB Infinity Cache, so every call streams them from HBM, as a decode step does.
Prints us/call and the weight-stream TB/s."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336),
                 "head": (128256, 4096)},
          "70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672)}}


def timed(fn, ws, iters):
    for w in ws[:2]:
        fn(w)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(iters):
        fn(ws[i % len(ws)])
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / iters


def main():
    from mxllm.ops import _ext

    nat = _ext.native()
    models = sys.argv[1].split(",") if len(sys.argv) > 1 else ["8b", "70b"]
    out = {}
    for model in models:
        for name, (N, K) in SHAPES[model].items():
            nbytes = N * K * 2
            copies = max(2, (600 << 20) // nbytes + 1)
            ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
            for M in (1, 4, 8, 16, 32, 64):
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                tb = timed(lambda w: F.linear(x, w), ws, 3 * copies)
                rec = {"blaslt_us": round(tb, 1), "blaslt_TBs": round(nbytes / tb / 1e6, 2)}
                if M <= 32:  # the HIP kernel's row limit
                    th = timed(lambda w: nat.skinny_linear(x, w), ws, 3 * copies)
                    rec.update(hip_us=round(th, 1), hip_TBs=round(nbytes / th / 1e6, 2))
                out[f"{model}/{name}/M{M}"] = rec
                print(json.dumps({f"{model}/{name}/M{M}": out[f"{model}/{name}/M{M}"]}), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
