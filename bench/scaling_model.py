#!/usr/bin/env python3
"""Calibrated 1/2/4/8-GPU projection of the data-parallel fine-tune benchmarks
(the GPU pool offers one MI355X; the 8-GPU curve is measured by
the driver at round end).  PROJECTION, not measurement.

Inputs: the measured one-GPU step (bench JSON), the measured fraction of the
step spent in backward (roctx ranges of profiles/r1b_70b_lora_roctx_ranges.md:
~2/3), the gradient bytes each step all-reduces, and an assumed achieved
all-reduce bus bandwidth over xGMI (two cases: 150 GB/s = one ring bound to one
153 GB/s link; 350 GB/s = RCCL multi-channel rings over several links).
Model per step at N ranks:
  ring bytes per GPU  = 2 (N-1)/N * grad_bytes
  comm time           = ring bytes / bus bandwidth
  exposed             = max(0, comm - backward_time + last_bucket_time) ... the
                        buckets fire during backward, only what outlasts it
                        (plus the last bucket, launched when backward ends)
                        adds to the step
  step(N)             = step(1) * (1 + contention) + exposed
``contention`` (RCCL kernels occupying CUs while GEMMs run) is taken as 2 %.
"""
from __future__ import annotations

import argparse
import json


def project(step_ms: float, tokens_per_gpu: int, grad_bytes: float, bw_gbs: float, bucket_mb: float = 128.0,
            bwd_frac: float = 0.66, contention: float = 0.02):
    rows = []
    for n in (1, 2, 4, 8):
        if n == 1:
            rows.append({"n": n, "ms": step_ms, "tok_s": tokens_per_gpu * 1e3 / step_ms, "exposed_ms": 0.0})
            continue
        ring = 2.0 * (n - 1) / n
        comm = ring * grad_bytes / (bw_gbs * 1e9) * 1e3
        last = ring * min(bucket_mb * 2 ** 20, grad_bytes) / (bw_gbs * 1e9) * 1e3
        exposed = max(0.0, comm - bwd_frac * step_ms) + last
        ms = step_ms * (1 + contention) + exposed
        rows.append({"n": n, "ms": ms, "tok_s": n * tokens_per_gpu * 1e3 / ms, "exposed_ms": exposed})
    for r in rows:
        r["efficiency"] = r["tok_s"] / (rows[0]["tok_s"] * r["n"])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    cases = {
        "Llama-3.1-70B LoRA r=16 DDP (headline), 613 MB bf16 adapter grads":
            dict(step_ms=1026.2, tokens_per_gpu=4096, grad_bytes=306_708_480 * 2),
        "Llama-3.1-8B full fine-tune DDP, 16.06 GB bf16 grads":
            dict(step_ms=217.7, tokens_per_gpu=4096, grad_bytes=8.03e9 * 2),
    }
    out = {}
    for name, kw in cases.items():
        out[name] = {f"{bw} GB/s": project(bw_gbs=bw, **kw) for bw in (150, 350)}
    if a.json:
        print(json.dumps(out))
        return
    for name, d in out.items():
        print(f"### {name}\n")
        print("| GPUs | bus bw | ms/step | tokens/s (node) | exposed comm ms | efficiency |")
        print("|---|---|---|---|---|---|")
        for bw, rows in d.items():
            for r in rows:
                print(f"| {r['n']} | {bw} | {r['ms']:.1f} | {r['tok_s']:,.0f} | {r['exposed_ms']:.1f} | "
                      f"{r['efficiency']:.3f} |")
        print()


if __name__ == "__main__":
    main()
