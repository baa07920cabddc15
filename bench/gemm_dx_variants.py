"""dX = dY @ W variants for frozen-weight backward (W stored [N_out, K_in]).

(a) dy @ w                      (NN for hipBLASLt)
(b) (w.t() @ dy.t()).t()        (operand-swapped; result transposed view)
(c) (b) + .contiguous()         (materialised)
(d) addmm_ into C (beta=1)      (the LoRA-fused form)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxllm.utils import gemm_tuning  # noqa: E402


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


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "table":
        gemm_tuning.enable()
    M = 4096
    for name, (N, K) in {"gu": (57344, 8192), "down": (8192, 28672), "o": (8192, 8192), "qkv": (10240, 8192),
                         "head": (128256, 8192)}.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        c = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        r = {"a_nn": fl / timeit(lambda: dy @ w) / 1e9,
             "b_swapped_view": fl / timeit(lambda: (w.t() @ dy.t()).t()) / 1e9,
             "c_swapped_contig": fl / timeit(lambda: (w.t() @ dy.t()).t().contiguous()) / 1e9,
             "d_addmm_beta1": fl / timeit(lambda: c.addmm_(dy, w)) / 1e9}
        print(json.dumps({"shape": name, "TF": {k: round(v, 1) for k, v in r.items()}}), flush=True)
        del w, dy, c


if __name__ == "__main__":
    main()
