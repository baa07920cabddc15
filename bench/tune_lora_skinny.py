"""Tune (PyTorch TunableOp) the memory-bound LoRA GEMMs of the 70B step with the
exact operand layouts _LoRAAugFn uses, then A/B them against the default choice.

Per projection (T = 4096, pad 64, R = n*r):
  t  : x_aug[:, K:]   = s * x  @ A_pad^T      (x, out: row stride K+64)
  g  : dy_aug[:, N:]  = s * dy @ B_pad        (dy, out: row stride N+64)
  dA : gA            += g^T @ x               (g: row stride N+64, x: K+64)
  dB : gB_i          += dy_i^T @ (s t_i)      (dy_i: N+64, t_i: K+64, out: row stride R)
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINEARS = {"qkv": (8192, [8192, 1024, 1024]), "o": (8192, [8192]), "gu": (8192, [28672, 28672]),
           "down": (28672, [8192])}
T, PAD, r = 4096, 64, 16


def timeit(fn, iters=20):
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


def ops_for(K, splits):
    bf = torch.bfloat16
    N, R = sum(splits), r * len(splits)
    wbuf = torch.randn(N + PAD, K + PAD, device="cuda", dtype=bf) * 0.02
    xa = torch.randn(T, K + PAD, device="cuda", dtype=bf)
    dya = torch.randn(T, N + PAD, device="cuda", dtype=bf)
    ga = torch.zeros(R, K, device="cuda", dtype=bf)
    gb = torch.zeros(N, R, device="cuda", dtype=bf)
    x2, st, dy2, g = xa[:, :K], xa[:, K:K + R], dya[:, :N], dya[:, N:N + R]
    fns = {"t": lambda: xa[:, K:].addmm_(x2, wbuf[N:, :K].t(), beta=0.0, alpha=2.0),
           "g": lambda: dya[:, N:].addmm_(dy2, wbuf[:N, K:], beta=0.0, alpha=2.0),
           "dA": lambda: ga.addmm_(g.t(), x2)}

    def db():
        off = 0
        for i, n_i in enumerate(splits):
            gb[off:off + n_i, i * r:(i + 1) * r].addmm_(dy2[:, off:off + n_i].t(), st[:, i * r:(i + 1) * r])
            off += n_i

    fns["dB"] = db
    return fns


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tunableop_lora_skinny.csv"))
    ap.add_argument("--max-ms", type=int, default=30)
    ap.add_argument("--linears", default="qkv,o,gu,down")
    a = ap.parse_args()
    tun = torch.cuda.tunable
    for name in a.linears.split(","):
        K, splits = LINEARS[name]
        fns = ops_for(K, splits)
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
        print(json.dumps({name: {"default_ms": {k: round(v, 4) for k, v in base.items()},
                                 "tuned_ms": {k: round(v, 4) for k, v in tuned.items()},
                                 "tune_s": round(time.time() - t0, 1)}}), flush=True)
        del fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
