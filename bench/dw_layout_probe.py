"""Full fine-tuning weight-gradient GEMM: which operand layout is faster?

dW[N, K] += dy[T, N]^T @ x[T, K] reduces over the token dimension T, but both
activations are stored token-major (contiguous along N / K), so hipBLASLt runs
its "NT" kernel family with both operands reduction-strided.  Alternative:
transpose dy and x into token-contiguous images first (one memory-bound pass
over each activation) and run the reduction-contiguous "TN" GEMM, the same
kernel family as the forward projection.

Measures, per Llama-3.1 projection (T = 4096 tokens), with the repo's tuned
solution table enabled:
  nt          g.addmm_(dy.t(), x)                       (current)
  tn_gemm     g.addmm_(dyT, xT.t())                     (GEMM only)
  tn_total    transpose(dy), transpose(x) + tn_gemm
Prints one JSON line per (model, projection).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (K in, N out)
    "70b": {"qkv": (8192, 10240), "o": (8192, 8192), "gu": (8192, 57344), "down": (28672, 8192),
            "head": (8192, 128256)},
    "8b": {"qkv": (4096, 6144), "o": (4096, 4096), "gu": (4096, 28672), "down": (14336, 4096),
           "head": (4096, 128256)},
}
T = 4096


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="70b,8b")
    ap.add_argument("--native", action="store_true", help="use mxllm's HIP transpose kernel")
    a = ap.parse_args()
    from mxllm.utils import gemm_tuning

    gemm_tuning.enable()
    tr = (lambda t: t.t().contiguous())
    if a.native:
        from mxllm import ops

        tr = ops.transpose2d
    for m in a.models.split(","):
        for name, (K, N) in SHAPES[m].items():
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
            g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
            xT, dyT = tr(x), tr(dy)
            fl = 2.0 * T * N * K
            ms = {"nt": timeit(lambda: g.addmm_(dy.t(), x)),
                  "tn_gemm": timeit(lambda: g.addmm_(dyT, xT.t())),
                  "transpose": timeit(lambda: (tr(dy), tr(x)))}
            ms["tn_total"] = ms["tn_gemm"] + ms["transpose"]
            tf = {k: round(fl / v / 1e9, 1) for k, v in ms.items() if k != "transpose"}
            print(json.dumps({"model": m, "proj": name, "ms": {k: round(v, 4) for k, v in ms.items()}, "TF": tf,
                              "transpose_GBps": round(4 * T * (N + K) / ms["transpose"] / 1e6, 1)}), flush=True)
            del x, dy, g, xT, dyT


if __name__ == "__main__":
    main()
