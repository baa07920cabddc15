"""FP8 (OCP e4m3) weight-only quantisation for serving (MI355X / gfx950).

Decode is bound by streaming every projection weight once per step (the bf16
GEMMs already run at ~5.6 TB/s), so 1-byte weights roughly halve the step time
of the memory-bound phase and the weight footprint (70B: 141 -> 70 GB, leaving
more HBM for the KV cache).  Activations stay bf16; the HIP kernel
(``csrc/kernels/fp8_gemm.hip``) dequantises 16 weights per lane in registers and
feeds bf16 MFMAs, and applies the per-output-channel scale in its epilogue.

Format: per output channel n, ``scale[n] = amax(|W[n, :]|) / 448`` and
``q[n, k] = e4m3(W[n, k] / scale[n])`` (round to nearest even, saturating).
Codes whose exponent field would be 0 (zero and subnormals, |W/scale| < 2^-6)
are stored as the smallest normal of the same sign: that error is at most
2^-6 * scale (<= 1/28672 of the row's largest weight) and it lets the kernel
decode every byte with four integer ALU operations and no special cases.

Up to ``SMALL_M`` tokens per call (small decode batches) the projection runs on the
weight-only HIP kernel with bf16 activations; larger calls quantise the activations
per token as well and use hipBLASLt's fp8 GEMM (``torch._scaled_mm``, row-wise
scales).  Training never uses this path (the fine-tuning benchmark is bf16 end to
end).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops._ext import native, use_native

E4M3_MAX = 448.0
# Calls of up to SMALL_M tokens use the weight-only HIP kernel (bf16 activations, the fp8
# weights streamed once per call); larger calls quantise the activations per token too
# and run hipBLASLt's fp8 MFMA GEMM (W8A8).  The threshold is aligned to the graphed
# decode's power-of-two batch buckets (mxllm/serve/engine.py), which is where it was
# measured (70B decode step, archive/profiles/r1g_fp8_decode_ab.md): the 8-row bucket 21.1 ms on
# the HIP kernel vs 27.7 ms on hipBLASLt, the 16-row bucket (9..16 live sequences; the
# profile's "12 tokens" row also ran 16-row GEMMs) 25.2 vs 24.6 ms.  Eager calls with 9..15
# rows were not measured separately.  Decode accuracy of both routings at the 16-row
# bucket: tests/test_model_gpu.py::test_engine_fp8_graphed_decode_b16_close_to_bf16.
SMALL_M = int(os.environ.get("MXLLM_W8_SMALL_M", "8"))


def quantize_e4m3(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """w [N, K] -> (codes uint8 [N, K], scale f32 [N])."""
    wf = w.float()
    amax = wf.abs().amax(dim=1).clamp_min(1e-30)
    scale = amax / E4M3_MAX
    v = (wf / scale[:, None]).clamp_(-E4M3_MAX, E4M3_MAX)
    q = v.to(torch.float8_e4m3fn).view(torch.uint8)
    exp0 = (q & 0x78) == 0  # zero or subnormal -> smallest normal, same sign
    q = torch.where(exp0, (q & 0x80) | 0x08, q)
    return q.contiguous(), scale.contiguous()


def dequantize_e4m3(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """Reference decode (fp32) of codes produced by :func:`quantize_e4m3`."""
    qi = q.to(torch.int32)
    e = (qi >> 3) & 0xF
    m = (qi & 7).float()
    mag = torch.ldexp(1.0 + m / 8.0, e - 7)
    v = torch.where((qi & 0x80) != 0, -mag, mag)
    return v * scale.float()[:, None]


class W8Linear(nn.Module):
    """Frozen projection y = x W^T with fp8 weights (serving only)."""

    def __init__(self, weight: torch.Tensor):
        super().__init__()
        q, s = quantize_e4m3(weight.detach())
        self.register_buffer("q", q)
        self.register_buffer("scale", s)
        self.out_features, self.in_features = q.shape

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x2 = x.reshape(-1, self.in_features)
        if x2.stride(1) != 1 or x2.stride(0) % 8:
            x2 = x2.contiguous()  # the HIP kernels take 16-B-aligned rows
        M = x2.shape[0]
        if not use_native(x2):
            y = torch.matmul(x2, dequantize_e4m3(self.q, self.scale).to(x2.dtype).t())
        elif M <= SMALL_M or self.in_features % 16:
            # weight-streaming HIP kernel: bf16 activations, weights dequantised in registers
            # (it falls back to dequantise + hipBLASLt for shapes it does not take)
            y = native().w8_linear(x2, self.q, self.scale)
        else:
            # larger batches / prefill: fp8 x fp8 MFMA GEMM (hipBLASLt), per-token activation
            # scales and the per-channel weight scales applied by the GEMM epilogue
            xq, sa = native().quant_rows_e4m3(x2)  # one HIP pass
            y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), self.q.view(torch.float8_e4m3fn).t(), scale_a=sa,
                                 scale_b=self.scale.view(1, -1), out_dtype=x2.dtype)
        return y.view(*x.shape[:-1], self.out_features)


@torch.no_grad()
def quantize_model_fp8_(model) -> int:
    """Replace every transformer projection (qkv, o, gate/up, down) of a Llama by
    a :class:`W8Linear` (LoRA adapters are merged first).  Embedding, norms and
    the LM head stay bf16.  Returns the number of weight bytes saved."""
    from ..models.llama import FusedLinear
    from .engine import merge_lora_

    merge_lora_(model)
    saved = 0
    for layer in model.layers:
        for name in ("wqkv", "wo", "wgu", "wd"):
            lin = getattr(layer, name)
            if isinstance(lin, FusedLinear):
                w = lin.weight
                setattr(layer, name, W8Linear(w))
                saved += w.numel() * (w.element_size() - 1)
                del lin, w
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return saved
