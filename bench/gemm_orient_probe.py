"""Which storage orientation of a LoRA-augmented projection weight is faster
over one training step (forward y = x W^T + input-gradient dx = dy W)?

  row-major W [N, K] (current):   fwd x @ W^T  (hipBLASLt "TN"),  dx dy @ W   ("NN")
  transposed Wt = W^T [K, N]:     fwd x @ Wt   ("NN"),            dx dy @ Wt^T ("TN")

Llama-3.1-70B shapes at 4096 tokens, LoRA-augmented (pad 64 on both sides), tuned GEMM
table on.  Prints ms per GEMM and per (fwd + dx) pair for both orientations."""
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
    gemm_tuning.enable()
    T, pad = 4096, 64
    shapes = {"qkv": (8192, 10240), "o": (8192, 8192), "gu": (8192, 57344), "down": (28672, 8192)}
    res = {}
    for name, (K, N) in shapes.items():
        Kp, Np = K + pad, N + pad
        w = torch.randn(Np, Kp, device="cuda", dtype=torch.bfloat16) * 0.02   # wbuf [[W, B], [A, 0]]
        wt = w.t().contiguous()                                                 # [[W^T, A^T], [B^T, 0]]
        x = torch.randn(T, Kp, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, Np, device="cuda", dtype=torch.bfloat16)
        r = {"fwd_rowmajor": timeit(lambda: torch.mm(x, w[:N, :].t())),
             "dx_rowmajor": timeit(lambda: torch.mm(dy, w[:, :K])),
             "fwd_transposed": timeit(lambda: torch.mm(x, wt[:, :N])),
             "dx_transposed": timeit(lambda: torch.mm(dy, wt[:K, :].t()))}
        r["pair_rowmajor"] = r["fwd_rowmajor"] + r["dx_rowmajor"]
        r["pair_transposed"] = r["fwd_transposed"] + r["dx_transposed"]
        fl = 2.0 * T * Kp * N
        r["fwd_tf"] = [round(fl / r["fwd_rowmajor"] / 1e9), round(fl / r["fwd_transposed"] / 1e9)]
        res[name] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        print(json.dumps({name: res[name]}), flush=True)
        del w, wt, x, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
