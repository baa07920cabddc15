"""dW = dy^T x (token-major operands) at the Llama-3.1 projection shapes: the hand-written MFMA
kernel (csrc/kernels/dw_gemm.hip) vs the HIP transpose + hipBLASLt "TN" path and the direct
hipBLASLt "NT" GEMM.  One JSON line per (model, projection, output dtype).

  python bench/dw_gemm_probe.py [--models 8b,70b] [--T 4096] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # projection: (M = out features, N = in features)
    "8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336), "head": (128256, 4096)},
    "70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gu": (57344, 8192), "down": (8192, 28672)},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="8b,70b")
    ap.add_argument("--T", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--f32", action="store_true", help="fp32 output with beta 1 (ZeRO-3 / fp32 grads)")
    a = ap.parse_args()
    import torch

    from mxllm.ops import native
    from mxllm.ops.linear import transpose2d
    from mxllm.utils import gemm_tuning

    gemm_tuning.enable()
    dev = torch.device("cuda", 0)
    odt = torch.float32 if a.f32 else torch.bfloat16
    beta = 1.0 if a.f32 else 0.0

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    for model in a.models.split(","):
        for proj, (M, N) in SHAPES[model].items():
            torch.manual_seed(0)
            dy = torch.randn(a.T, M, device=dev, dtype=torch.bfloat16)
            x = torch.randn(a.T, N, device=dev, dtype=torch.bfloat16)
            out_k = torch.zeros(M, N, device=dev, dtype=odt)
            out_t = torch.zeros(M, N, device=dev, dtype=odt)
            out_n = torch.zeros(M, N, device=dev, dtype=odt)

            def kern():
                os.environ["MXLLM_DW_GEMM"] = "dbuf"
                assert native().dw_gemm(dy, x, out_k, beta, None)

            def ring():
                os.environ["MXLLM_DW_GEMM"] = "ring"
                assert native().dw_gemm(dy, x, out_k, beta, None)

            def w8():
                os.environ["MXLLM_DW_GEMM"] = "w8"
                assert native().dw_gemm(dy, x, out_k, beta, None)

            def tn():
                xt, dyt = transpose2d(x), transpose2d(dy)
                if a.f32:
                    torch.ops.aten.addmm.dtype_out(out_t, dyt, xt.t(), torch.float32, beta=beta, out=out_t)
                else:
                    out_t.addmm_(dyt, xt.t(), beta=beta)

            def nt():
                if a.f32:
                    torch.ops.aten.addmm.dtype_out(out_n, dy.t(), x, torch.float32, beta=beta, out=out_n)
                else:
                    out_n.addmm_(dy.t(), x, beta=beta)

            res = {}
            for name, fn in (("kernel", kern), ("ring", ring), ("w8", w8), ("tn_total", tn), ("nt", nt)):
                res[name] = timeit(fn)
            # numerics after one call each from zero
            err = {}
            for name, fn in (("kernel", kern), ("ring", ring), ("w8", w8)):
                out_k.zero_(), out_t.zero_()
                fn(), tn()
                torch.cuda.synchronize()
                err[name] = ((out_k.float() - out_t.float()).norm() / out_t.float().norm()).item()
            fl = 2.0 * a.T * M * N
            print(json.dumps({"model": model, "proj": proj, "M": M, "N": N, "T": a.T, "out": str(odt).split(".")[-1],
                              "ms": {k: round(v, 4) for k, v in res.items()},
                              "TF": {k: round(fl / v / 1e9, 1) for k, v in res.items()},
                              "rel_err_vs_tn": err}), flush=True)
            del dy, x, out_k, out_t, out_n
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
