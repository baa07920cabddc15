"""First GPU probe: extension loads, RMSNorm numerics, hipBLASLt GEMM rates at
the Llama-3.1-70B/8B projection shapes, HBM capacity.  Prints JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / iters


def main():
    dev = torch.device("cuda", 0)
    free, total = torch.cuda.mem_get_info()
    print(json.dumps({"probe": "mem", "free_gb": free / 1e9, "total_gb": total / 1e9,
                      "name": torch.cuda.get_device_name(0)}), flush=True)
    torch.ops.load_library(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mxllm", "_C.so"))
    T, H = 4096, 8192
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(H, device=dev, dtype=torch.bfloat16)
    y, rstd, _ = torch.ops.mxllm.rmsnorm_fwd(x, None, w, 1e-5)
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    err = (y.float() - ref).abs().max().item()
    ms = timeit(lambda: torch.ops.mxllm.rmsnorm_fwd(x, None, w, 1e-5))
    print(json.dumps({"probe": "rmsnorm_fwd", "max_err": err, "ms": ms,
                      "GBps": 2 * T * H * 2 / ms / 1e6}), flush=True)
    dy = torch.randn_like(x)
    ms = timeit(lambda: torch.ops.mxllm.rmsnorm_bwd(dy, x, w, rstd, None, True))
    print(json.dumps({"probe": "rmsnorm_bwd", "ms": ms, "GBps": 3 * T * H * 2 / ms / 1e6}), flush=True)

    shapes = {
        "70b_qkv": (4096, 8192, 10240), "70b_o": (4096, 8192, 8192), "70b_gu": (4096, 8192, 57344),
        "70b_down": (4096, 28672, 8192), "70b_head": (4096, 8192, 128256),
        "8b_qkv": (4096, 4096, 6144), "8b_gu": (4096, 4096, 28672), "8b_down": (4096, 14336, 4096),
    }
    for name, (M, K, N) in shapes.items():
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        g = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        ms_f = timeit(lambda: torch.nn.functional.linear(a, W), iters=10)
        ms_b = timeit(lambda: g @ W, iters=10)  # dX = dY W
        ms_w = timeit(lambda: g.t() @ a, iters=10)  # dW = dY^T X
        print(json.dumps({"probe": "gemm", "shape": name, "MKN": [M, K, N],
                          "fwd_TF": fl / ms_f / 1e9, "dx_TF": fl / ms_b / 1e9, "dw_TF": fl / ms_w / 1e9}), flush=True)
        del a, W, g
    # torch SDPA for reference (aotriton; oracle only, never used by mxllm)
    try:
        B, Hq, S, D = 2, 64, 2048, 128
        q = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True), iters=10)
        fl = 4.0 * B * Hq * S * S * D / 2
        print(json.dumps({"probe": "sdpa_ref_fwd", "ms": ms, "TF": fl / ms / 1e9}), flush=True)
    except Exception as e:  # noqa
        print(json.dumps({"probe": "sdpa_ref_fwd", "error": str(e)[:200]}), flush=True)


if __name__ == "__main__":
    main()
