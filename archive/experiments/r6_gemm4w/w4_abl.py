"""Timing-only ablations of the 4-wave gemm kernel on the 70B-LoRA o-projection dX shape (NN, M4096 N8192
K8256): MXLLM_GEMM8_W4 = 1 real, 2 no DMA waits / no next-tile DMA, 3 no LDS reads, 4 no MFMAs, 5 no barrier, 6 MFMAs + barriers only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxllm.ops import native  # noqa: E402

ops = native()
dev = torch.device("cuda", 0)
M, N, K = 4096, 8192, 8256
a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
b = (torch.rand(K, N + 64, device=dev) * 2 - 1).bfloat16()[:, :N]
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for v in ("0", "1", "2", "3", "4", "5", "6"):
    if v == "0":
        os.environ.pop("MXLLM_GEMM8_W4", None)
        os.environ["MXLLM_GEMM8_PH"] = "4"
    else:
        os.environ.pop("MXLLM_GEMM8_PH", None)
        os.environ["MXLLM_GEMM8_W4"] = v
    for _ in range(3):
        ops.gemm8(a, True, b, False, o, 0.0, None, 1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.gemm8(a, True, b, False, o, 0.0, None, 1.0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"W4={v}: {ms:.3f} ms  {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
