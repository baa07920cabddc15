"""Which storage of a frozen LoRA-augmented projection weight is faster overall?

Current: wbuf [N+p, K+p] row-major  -> forward x_aug @ wbuf^T is hipBLASLt "TN"
         (both operands reduction-contiguous), backward dX = dy_aug @ wbuf is "NN".
Swapped: wt = wbuf^T [K+p, N+p]      -> forward is "NN", backward dX is "TN".

Measures TFLOP/s of the four GEMMs per Llama-3.1-70B projection (T = 4096 tokens,
pad 64) with the library's default heuristics, then with TunableOp tuning of
every variant (--tune).  Prints one JSON line per projection.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PROJ = {"qkv": (8192, 10240), "o": (8192, 8192), "gu": (8192, 57344), "down": (28672, 8192)}
T, P = 4096, 64


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


def measure(names):
    out = {}
    for name in names:
        K, N = PROJ[name]
        wbuf = torch.randn(N + P, K + P, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = wbuf.t().contiguous()
        xa = torch.randn(T, K + P, device="cuda", dtype=torch.bfloat16)
        dya = torch.randn(T, N + P, device="cuda", dtype=torch.bfloat16)
        fl_f, fl_b = 2.0 * T * N * (K + P), 2.0 * T * K * (N + P)
        ms = {"cur_fwd_TN": timeit(lambda: torch.mm(xa, wbuf[:N, :].t())),
              "cur_bwd_NN": timeit(lambda: torch.mm(dya, wbuf[:, :K])),
              "swp_fwd_NN": timeit(lambda: torch.mm(xa, wt[:, :N])),
              "swp_bwd_TN": timeit(lambda: torch.mm(dya, wt[:K, :].t()))}
        tf = {k: round((fl_f if "fwd" in k else fl_b) / v / 1e9, 1) for k, v in ms.items()}
        out[name] = {"ms": {k: round(v, 4) for k, v in ms.items()}, "TF": tf,
                     "cur_total_ms": round(ms["cur_fwd_TN"] + ms["cur_bwd_NN"], 4),
                     "swp_total_ms": round(ms["swp_fwd_NN"] + ms["swp_bwd_TN"], 4)}
        del wbuf, wt, xa, dya
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proj", default="qkv,o,gu,down")
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--max-ms", type=int, default=150)
    a = ap.parse_args()
    names = a.proj.split(",")
    print(json.dumps({"phase": "default", "res": measure(names)}), flush=True)
    if a.tune:
        tun = torch.cuda.tunable
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(a.max_ms)
        tun.set_filename(os.path.join("/tmp", "swap_tune.csv"))
        measure(names)
        tun.tuning_enable(False)
        print(json.dumps({"phase": "tuned", "res": measure(names)}), flush=True)


if __name__ == "__main__":
    main()
