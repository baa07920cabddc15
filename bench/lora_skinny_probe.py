"""Per-call time of the LoRA rank-r GEMMs of one Llama-3.1-70B layer (T = 4096
tokens, rank 16 per split, pad 64) as issued by mxllm/ops/linear.py _LoRAAugFn:
  fwd  st  = s x A^T            (into the x_aug tail)
  bwd  g   = s dy B             (into the dy_aug tail)
       dA += g^T x              (bf16 grad, beta = 1)
       dB_i += dy_i^T st_i      (diagonal blocks)
with hipBLASLt (torch.mm / addmm_) and, if built, the native HIP kernels.
Reports us/call and the effective HBM bandwidth of the dominant operand."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

T, r, P = 4096, 16, 64
PROJ = {"qkv": (8192, [8192, 1024, 1024]), "o": (8192, [8192]), "gu": (8192, [28672, 28672]),
        "down": (28672, [8192])}


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
    return 1e3 * a.elapsed_time(b) / iters


def main():
    from mxllm.ops import _ext
    from mxllm.utils import gemm_tuning

    gemm_tuning.enable()
    nat = _ext.native() if _ext.available() else None
    has_native = nat is not None and hasattr(nat, "lora_xwt")
    dev = "cuda"
    tot = {"blas": 0.0, "hip": 0.0}
    for name, (K, splits) in PROJ.items():
        N, n = sum(splits), len(splits)
        R = n * r
        wbuf = torch.randn(N + P, K + P, device=dev, dtype=torch.bfloat16) * 0.02
        wbuf[N + R:, :] = 0
        wbuf[:, K + R:] = 0
        xa = torch.randn(T, K + P, device=dev, dtype=torch.bfloat16)
        dya = torch.randn(T, N + P, device=dev, dtype=torch.bfloat16)
        x2, dy2 = xa[:, :K], dya[:, :N]
        ga = torch.zeros(R, K, device=dev, dtype=torch.bfloat16)
        gb = torch.zeros(N, R, device=dev, dtype=torch.bfloat16)
        s = 2.0
        res = {"proj": name}
        res["fwd_st_blas"] = timeit(lambda: xa[:, K:].addmm_(x2, wbuf[N:, :K].t(), beta=0.0, alpha=s))
        res["bwd_g_blas"] = timeit(lambda: dya[:, N:].addmm_(dy2, wbuf[:N, K:], beta=0.0, alpha=s))
        g, st = dya[:, N:N + R], xa[:, K:K + R]
        res["dA_blas"] = timeit(lambda: ga.addmm_(g.t(), x2))

        def db_blas():
            off = 0
            for i, n_i in enumerate(splits):
                gb[off:off + n_i, i * r:(i + 1) * r].addmm_(dy2[:, off:off + n_i].t(), st[:, i * r:(i + 1) * r])
                off += n_i
        res["dB_blas"] = timeit(db_blas)
        res["blas_total"] = sum(v for k, v in res.items() if k.endswith("_blas"))
        tot["blas"] += res["blas_total"]
        if has_native:
            bt = wbuf[:N, K:].t().contiguous()
            res["fwd_st_hip"] = timeit(lambda: nat.lora_xwt(x2, wbuf[N:, :K], xa[:, K:], s))
            res["bwd_g_hip"] = timeit(lambda: nat.lora_xwt(dy2, bt, dya[:, N:], s))
            res["dAdB_hip"] = timeit(lambda: nat.lora_grads(x2, dy2, dya[:, N:], xa[:, K:], ga, gb, list(splits), r,
                                                            True))
            res["hip_total"] = sum(v for k, v in res.items() if k.endswith("_hip"))
            tot["hip"] += res["hip_total"]
        res["x_MB"], res["dy_MB"] = round(T * K * 2 / 1e6, 1), round(T * N * 2 / 1e6, 1)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
        del wbuf, xa, dya, ga, gb
    print(json.dumps({"layer_total_us": {k: round(v, 1) for k, v in tot.items()},
                      "step_ms_80_layers": {k: round(v * 80 / 1e3, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
