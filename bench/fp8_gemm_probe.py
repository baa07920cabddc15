"""Probe: FP8 (e4m3) weight GEMMs through torch._scaled_mm / hipBLASLt on gfx950
for decode-shaped problems (M = 1..64 tokens, Llama-3.1-70B projection sizes),
against the bf16 GEMM.  Decode is weight-streaming bound, so fp8 weights
should approach 2x."""
import json
import time

import torch


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


def main():
    dev = "cuda"
    f8 = torch.float8_e4m3fnuz if hasattr(torch, "float8_e4m3fnuz") else torch.float8_e4m3fn
    for f8t in (torch.float8_e4m3fn, getattr(torch, "float8_e4m3fnuz", None)):
        if f8t is None:
            continue
        try:
            a = torch.randn(16, 256, device=dev).to(f8t)
            b = torch.randn(512, 256, device=dev).to(f8t)
            one = torch.ones((), device=dev)
            torch._scaled_mm(a, b.t(), one, one, out_dtype=torch.bfloat16)
            f8 = f8t
            print(json.dumps({"fp8_dtype_ok": str(f8t)}), flush=True)
            break
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"fp8_dtype_fail": str(f8t), "err": str(e)[:300]}), flush=True)
    for name, (K, N) in {"qkv": (8192, 10240), "o": (8192, 8192), "gu": (8192, 57344), "down": (28672, 8192)}.items():
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        w8 = w.float().to(f8)
        for M in (1, 8, 32, 64, 256):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            x8 = x.float().to(f8)
            one = torch.ones((), device=dev)
            rs_a = torch.ones(M, 1, device=dev)
            rs_b = torch.ones(1, N, device=dev)
            r = {"proj": name, "M": M, "bf16_us": round(1e3 * timeit(lambda: torch.mm(x, w.t())), 1)}
            try:
                r["fp8_tensorwise_us"] = round(1e3 * timeit(
                    lambda: torch._scaled_mm(x8, w8.t(), one, one, out_dtype=torch.bfloat16)), 1)
            except Exception as e:  # noqa: BLE001
                r["fp8_tensorwise_err"] = str(e)[:200]
            try:
                r["fp8_rowwise_us"] = round(1e3 * timeit(
                    lambda: torch._scaled_mm(x8, w8.t(), rs_a, rs_b, out_dtype=torch.bfloat16)), 1)
            except Exception as e:  # noqa: BLE001
                r["fp8_rowwise_err"] = str(e)[:200]
            r["weight_MB"] = round(N * K * 2 / 1e6, 1)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
