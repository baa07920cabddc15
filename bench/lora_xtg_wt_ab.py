#!/usr/bin/env python3
"""A/B of ``lora_xtg``'s wave-owns-tile mode (MXLLM_LORA_XTG_WT=1: each wave streams one 64-column tile
over all T rows, 4 adjacent tiles per workgroup) against the default (the 4 waves of a workgroup
split one tile's rows), at the Llama-3.1-70B headline shapes (T 4096, r 16): microseconds per
``lora_grads`` launch, alternating the two modes over ``--rounds``, plus the max relative difference
of their outputs.  Usage: python bench/lora_xtg_wt_ab.py [--rounds 6] [--calls 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.ops import native  # noqa: E402

PROJ = {"qkv": (8192, [8192, 1024, 1024]), "o": (8192, [8192]), "gu": (8192, [28672, 28672]),
        "down": (28672, [8192])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--wgs", default="256", help="MXLLM_LORA_WGS")
    ap.add_argument("--wt-min", default="1024", help="MXLLM_LORA_XTG_WT_MIN: tiles a launch needs for the wave-tile form")
    a = ap.parse_args()
    os.environ["MXLLM_LORA_WGS"] = a.wgs
    os.environ["MXLLM_LORA_XTG_WT_MIN"] = a.wt_min
    dev = torch.device("cuda", 0)
    ops = native()
    T, r, pad = a.tokens, 16, 64
    for name, (K, splits) in PROJ.items():
        N, R = sum(splits), r * len(splits)
        xa = torch.randn(T, K + pad, device=dev, dtype=torch.bfloat16)
        dya = torch.randn(T, N + pad, device=dev, dtype=torch.bfloat16)
        x2, dy2, g, st = xa[:, :K], dya[:, :N], dya[:, N:], xa[:, K:]
        res = {}
        times = {"0": [], "1": []}
        for _ in range(a.rounds):
            for wt in ("0", "1"):
                os.environ["MXLLM_LORA_XTG_WT"] = wt
                ga = torch.zeros(R, K, device=dev, dtype=torch.bfloat16)
                gb = torch.zeros(N, R, device=dev, dtype=torch.bfloat16)
                for _ in range(3):
                    ops.lora_grads(x2, dy2, g, st, ga, gb, splits, r, False)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.calls)]
                for s0, e0 in ev:
                    s0.record()
                    ops.lora_grads(x2, dy2, g, st, ga, gb, splits, r, False)
                    e0.record()
                torch.cuda.synchronize()
                times[wt].append(1e3 * statistics.median(s0.elapsed_time(e0) for s0, e0 in ev))
                res[wt] = (ga.float(), gb.float())
        diff = max(float((res["0"][i] - res["1"][i]).abs().max() / res["0"][i].abs().max().clamp_min(1e-30))
                   for i in range(2))
        gbytes = (T * (K + N) * 2 + T * R * 2 * 2) / 1e9
        line = {"proj": name, "ntiles": (K + N) // 64, "gb": round(gbytes, 3),
                "us_default": round(min(times["0"]), 1), "us_wave_tile": round(min(times["1"]), 1),
                "us_default_all": [round(t, 1) for t in times["0"]], "us_wave_tile_all": [round(t, 1) for t in times["1"]],
                "max_rel_diff": diff}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
