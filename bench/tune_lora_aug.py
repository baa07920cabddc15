"""Tune hipBLASLt/rocBLAS solutions (PyTorch TunableOp) for the LoRA-augmented
main GEMMs of the 70B training step, with the exact operand layouts the step
uses (row strides K+64 / N+64), and append them to the selection table.

  fwd: y  = x_aug[T, K+64] @ wbuf[:N, :]^T        (wbuf row stride K+64)
  bwd: dx = dy_aug[T, N+64] @ wbuf[:, :K]         (row stride K+64)
  bwd_tn: dx = dy_aug @ wxt^T  (wxt = [W; A]^T image: qkv and down projections by default)

The table is written after every shape, so a time limit loses at most one.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672)}
T, PAD = 4096, 64


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


def ops_for(N, K):
    bf = torch.bfloat16
    wbuf = torch.randn(N + PAD, K + PAD, device="cuda", dtype=bf) * 0.02
    xa = torch.randn(T, K + PAD, device="cuda", dtype=bf)
    dya = torch.randn(T, N + PAD, device="cuda", dtype=bf)
    wf, wb = wbuf[:N, :], wbuf[:, :K]
    wxt = wb.t().contiguous()  # FusedLinear.wxt: transposed [W; A] image (TN dX)
    return {"fwd": lambda: torch.mm(xa, wf.t()), "bwd": lambda: torch.mm(dya, wb),
            "bwd_tn": lambda: torch.mm(dya, wxt.t())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tunableop_lora_aug.csv"))
    ap.add_argument("--max-ms", type=int, default=60)
    ap.add_argument("--shapes", default="qkv,o,gu,down")
    ap.add_argument("--ops", default="fwd,bwd,bwd_tn", help="subset of fwd,bwd,bwd_tn to tune")
    a = ap.parse_args()
    tun = torch.cuda.tunable
    res = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        fns = {k: f for k, f in ops_for(N, K).items() if k in a.ops.split(",")}
        base = {k: timeit(f) for k, f in fns.items()}
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(a.max_ms)
        tun.set_filename(a.out)
        t0 = time.time()
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        if hasattr(tun, "write_file"):
            tun.write_file(a.out)
        tun.tuning_enable(False)
        tuned = {k: timeit(f) for k, f in fns.items()}
        tun.enable(False)
        res[name] = {"default_ms": {k: round(v, 4) for k, v in base.items()},
                     "tuned_ms": {k: round(v, 4) for k, v in tuned.items()}, "tune_s": round(time.time() - t0, 1)}
        print(json.dumps({name: res[name]}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
