#!/usr/bin/env python3
"""gemm8 phase timing from in-kernel cycle stamps (diagnostic build, MXLLM_GEMM8_STAMPS=8|4).

Runs the NN form at the 70B o-projection dX shape (M 4096, N 8192, K 8192 -> 512 tiles, 64 K-loop
iterations of 2 K-tiles) on uniform random data, after >= 2 s of warm-up launches, then reads the
stamps of the last launch: per workgroup (lane 0 of waves 0 / 4) the prologue, every K-loop
iteration, the loop end and the epilogue end.  Reports cycles per iteration against the MFMA floor
(2 waves x 128 v_mfma_f32_16x16x32_bf16 x 16 cycles = 4096 per SIMD per iteration), prologue and
epilogue cycles, and the clock (d memtime / d realtime x 100 MHz)."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.ops import native  # noqa: E402

NST = 80


def run(ph: str, M=4096, N=8192, K=8192):
    ops = native()
    dev = torch.device("cuda", 0)
    a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    os.environ["MXLLM_GEMM8_STAMPS"] = ph
    t0 = time.time()
    n = 0
    while time.time() - t0 < 2.0:
        ops.gemm8(a, True, b, False, o, 0.0, None, 1.0)
        n += 1
        if n % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    os.environ.pop("MXLLM_GEMM8_STAMPS")
    st = ops.gemm8_stamps()
    grid = (M // 256) * (N // 256)
    nit = (K // 64 + 1) // 2
    it, pro, epi, clk, loop, starts = [], [], [], [], [], []
    for wg in range(grid):
        for r in range(2):
            s = st[wg, r].tolist()
            t_start, rt_start, t_pro = s[0], s[1], s[2]
            its = s[3:3 + nit]
            t_loop, t_end, rt_end = s[NST - 3], s[NST - 2], s[NST - 1]
            starts.append(t_start)
            pro.append(t_pro - t_start)
            it.extend(b_ - a_ for a_, b_ in zip(its, its[1:]))
            loop.append(t_loop - t_pro)
            epi.append(t_end - t_loop)
            if rt_end > rt_start:
                clk.append((t_end - t_start) / (rt_end - rt_start) * 100.0)
    floor = 4096
    res = {"schedule_phases": int(ph), "shape": [M, N, K], "grid": grid, "launches_warm": n,
           "clock_mhz_median": round(statistics.median(clk), 1),
           "iter_cycles_median": statistics.median(it), "iter_cycles_p90": sorted(it)[int(0.9 * len(it))],
           "mfma_floor_per_iter": floor, "loop_mfma_util": round(floor / statistics.median(it), 3),
           "prologue_cycles_median": statistics.median(pro), "epilogue_cycles_median": statistics.median(epi),
           "loop_cycles_median": statistics.median(loop),
           "wg_start_spread_cycles": max(starts) - min(starts)}
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    out = [run(p) for p in (sys.argv[1:] or ["8", "4"])]
    if os.environ.get("STAMPS_JSON"):
        json.dump(out, open(os.environ["STAMPS_JSON"], "w"), indent=1)
