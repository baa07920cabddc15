#!/usr/bin/env python3
"""Calibrated 1/2/4/8-GPU projection of the data-parallel fine-tune benchmarks
(the GPU pool offers one MI355X; the 8-GPU curve is measured by
the driver at round end).  PROJECTION, not measurement.

Inputs: the measured one-GPU step (bench JSON), the measured fraction of the
step spent in backward (roctx ranges of archive/profiles/r1b_70b_lora_roctx_ranges.md:
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


def project_zero3(step_ms: float, tokens_per_gpu: int, param_bytes: float, bw_gbs: float, n: int = 8,
                  unit_bytes: float = 1.71e9, contention: float = 0.02):
    """BASELINE config 4 at n GPUs from the measured world-n EMULATED step (per-rank
    compute, memory traffic and shard sizes of the real run, no link traffic): per
    step every rank receives (n-1)/n of the model twice (forward + backward
    all-gathers) and sends it once (gradient reduce-scatter), overlapped with the
    compute (prefetch one unit ahead, asynchronous reduce-scatter); exposed = what
    outlasts the compute plus the first unit's gather."""
    comm = 3.0 * param_bytes * (n - 1) / n / (bw_gbs * 1e9) * 1e3
    first = unit_bytes * (n - 1) / n / (bw_gbs * 1e9) * 1e3
    exposed = max(0.0, comm - step_ms) + first
    ms = step_ms * (1 + contention) + exposed
    return {"n": n, "ms": ms, "tok_s": n * tokens_per_gpu * 1e3 / ms, "comm_ms": comm, "exposed_ms": exposed}


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
    z3 = {"act-ckpt, micro-batch 4 (bench default for config 4)": dict(step_ms=3726.1, tokens_per_gpu=8192),
          "no checkpointing, micro-batch 2": dict(step_ms=1570.8, tokens_per_gpu=4096)}
    z3_rows = {name: {f"{bw} GB/s": project_zero3(param_bytes=70.554e9 * 2, bw_gbs=bw, **kw) for bw in (150, 350)}
               for name, kw in z3.items()}
    if a.json:
        print(json.dumps({"ddp": out, "zero3_config4": z3_rows}))
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
    print("### Llama-3.1-70B FULL fine-tune, ZeRO-3, 8 GPUs (BASELINE config 4), from the world-8 emulated step\n")
    print("| config | bus bw | compute ms (measured, emulated) | comm ms | exposed ms | ms/step | tokens/s (node) |")
    print("|---|---|---|---|---|---|---|")
    for name, d in z3_rows.items():
        for bw, r in d.items():
            print(f"| {name} | {bw} | {z3[name]['step_ms']:.0f} | {r['comm_ms']:.0f} | {r['exposed_ms']:.0f} | "
                  f"{r['ms']:.0f} | {r['tok_s']:,.0f} |")
    print()


if __name__ == "__main__":
    main()
