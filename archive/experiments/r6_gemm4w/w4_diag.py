"""Where does the 4-wave gemm kernel (MXLLM_GEMM8_W4=1) go wrong?  Per operand order and K, the relative
error and the 16 x 16 output blocks (row block, col block) whose error exceeds bf16 level."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxllm.ops import native  # noqa: E402

os.environ["MXLLM_GEMM8_W4"] = "1"
ops = native()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
for a_kc, b_kc in ((True, True), (True, False), (False, True), (False, False)):
    for K in (64, 128, 192, 256, 640):
        M = N = 256
        a = (torch.rand((M, K) if a_kc else (K, M), device=dev, generator=g) * 2 - 1).bfloat16()
        b = (torch.rand((N, K) if b_kc else (K, N), device=dev, generator=g) * 2 - 1).bfloat16()
        A = a.float() if a_kc else a.float().t()
        B = b.float().t() if b_kc else b.float()
        ref = A @ B
        out = torch.empty(M, N, device=dev, dtype=torch.float32)
        ops.gemm8(a, a_kc, b, b_kc, out, 0.0, None, 1.0)
        err = ((out - ref).norm() / ref.norm()).item()
        d = (out - ref).abs().view(16, 16, 16, 16).amax(dim=(1, 3))  # [row block, col block]
        bad = (d > 1e-2 * ref.abs().max()).nonzero().tolist()
        print(f"a_kc={a_kc} b_kc={b_kc} K={K}: err {err:.2e}, bad blocks {len(bad)}: {bad[:12]}", flush=True)
