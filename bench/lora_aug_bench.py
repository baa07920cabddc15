"""LoRA GEMM layouts at the Llama-3.1-70B shapes (T = 4096 tokens).

current  : fwd  t = x A^T ; y = s t B^T (beta 0) ; y += x W^T (beta 1)
           bwd  dx = g A (beta 0) ; dx += dy W (beta 1)
K-aug    : one augmented weight buffer Wbuf [N+Rp, in+Rp] = [[W, sB], [A, 0]]
           fwd  y  = [x | t] @ Wbuf[:N, :]^T        (x_aug [T, in+Rp], t in the tail)
           bwd  dx = [dy | g] @ Wbuf[:, :in]        (dy_aug [T, N+Rp], g in the tail)
Prints ms per call for the main-GEMM part of each (the skinny t / g GEMMs are
the same in both layouts).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.utils import gemm_tuning  # noqa: E402


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
    if "table" in sys.argv[1:]:
        gemm_tuning.enable()
    T = 4096
    dev = "cuda"
    bf = torch.bfloat16
    for name, (N, K, n) in {"qkv": (10240, 8192, 3), "o": (8192, 8192, 1), "gu": (57344, 8192, 2),
                            "down": (8192, 28672, 1)}.items():
        R = 16 * n
        res = {"shape": name, "N": N, "K": K, "R": R}
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        a = torch.randn(R, K, device=dev, dtype=bf) * 0.02
        b = torch.randn(N, R, device=dev, dtype=bf) * 0.02
        x = torch.randn(T, K, device=dev, dtype=bf)
        t = torch.randn(T, R, device=dev, dtype=bf)
        dy = torch.randn(T, N, device=dev, dtype=bf)
        g = torch.randn(T, R, device=dev, dtype=bf)

        def cur_fwd():
            y = torch.empty(T, N, device=dev, dtype=bf)
            y.addmm_(t, b.t(), beta=0, alpha=2.0)
            y.addmm_(x, w.t())
            return y

        def cur_bwd():
            dx = torch.empty(T, K, device=dev, dtype=bf)
            dx.addmm_(g, a, beta=0)
            dx.addmm_(dy, w)
            return dx

        res["cur_fwd_ms"] = timeit(cur_fwd)
        res["cur_bwd_ms"] = timeit(cur_bwd)
        res["base_fwd_ms"] = timeit(lambda: x @ w.t())
        res["base_bwd_ms"] = timeit(lambda: dy @ w)
        for Rp in sorted({R, 64}):
            wbuf = torch.zeros(N + Rp, K + Rp, device=dev, dtype=bf)
            wbuf[:N, :K] = w
            wbuf[:N, K:K + R] = b
            wbuf[N:N + R, :K] = a
            xa = torch.zeros(T, K + Rp, device=dev, dtype=bf)
            xa[:, :K] = x
            xa[:, K:K + R] = t
            dya = torch.zeros(T, N + Rp, device=dev, dtype=bf)
            dya[:, :N] = dy
            dya[:, N:N + R] = g
            wf = wbuf[:N, :]
            wb = wbuf[:, :K]
            res[f"kaug{Rp}_fwd_ms"] = timeit(lambda: xa @ wf.t())
            res[f"kaug{Rp}_bwd_ms"] = timeit(lambda: dya @ wb)
            # numerics: K-aug == current up to bf16 rounding
            ref = cur_fwd().float()
            err = ((xa @ wf.t()).float() - ref).abs().max().item() / ref.abs().max().item()
            res[f"kaug{Rp}_fwd_relerr"] = err
            del wbuf, xa, dya
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        del w, a, b, x, t, dy, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
