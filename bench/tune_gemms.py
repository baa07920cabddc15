"""Tune hipBLASLt/rocBLAS solutions for the bench's GEMM shapes with PyTorch
TunableOp, write the selection table, and A/B it against the default choice.

The table lands in mxllm/tuning/tunableop_gfx950.csv and is loaded (tuning
off) by mxllm.utils.gemm_tuning.enable() — plain library GEMMs stay on
hipBLASLt/rocBLAS, we only pick the fastest of their own solutions per shape.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # (M, K, N) of y = x @ W^T at 4096 tokens
    "70b": [(4096, 8192, 10240), (4096, 8192, 8192), (4096, 8192, 57344), (4096, 28672, 8192),
            (4096, 8192, 128256)],
    "8b": [(4096, 4096, 6144), (4096, 4096, 4096), (4096, 4096, 28672), (4096, 14336, 4096),
           (4096, 4096, 128256)],
}


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def run_all(shapes, full):
    res = {}
    dev = "cuda"
    for (M, K, N) in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        c = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        cx = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        r = {"fwd": fl / timeit(lambda: torch.matmul(x, w.t())) / 1e9,
             "dx": fl / timeit(lambda: torch.matmul(dy, w)) / 1e9,
             "fwd_beta1": fl / timeit(lambda: c.addmm_(x, w.t())) / 1e9,
             "dx_beta1": fl / timeit(lambda: cx.addmm_(dy, w)) / 1e9}
        if full:
            r["dw"] = fl / timeit(lambda: torch.matmul(dy.t(), x)) / 1e9
        res[f"{M}x{K}x{N}"] = {k: round(v, 1) for k, v in r.items()}
        del x, w, dy, c, cx
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="70b,8b")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tunableop_gfx950.csv"))
    ap.add_argument("--max-ms", type=int, default=400)
    a = ap.parse_args()
    shapes = [s for m in a.models.split(",") for s in SHAPES[m]]
    base = run_all(shapes, True)
    print(json.dumps({"phase": "default", "TF": base}), flush=True)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_filename(a.out)
    t0 = time.time()
    run_all(shapes, True)
    tun.write_file(a.out)
    print(json.dumps({"phase": "tuning", "seconds": round(time.time() - t0, 1)}), flush=True)
    tun.tuning_enable(False)
    tuned = run_all(shapes, True)
    print(json.dumps({"phase": "tuned", "TF": tuned}), flush=True)


if __name__ == "__main__":
    main()
