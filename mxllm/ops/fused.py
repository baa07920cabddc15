"""Forward projections with their elementwise consumer fused into the GEMM epilogue.

VERDICT r4 item 5: in the 8B full fine-tune (BASELINE config 2) the forward's memory-bound
passes -- RoPE + head split (``rope_split``) after the qkv projection, SwiGLU after the
gate-up projection -- ran 3.6-11x off their rooflines because the overlapped AdamW saturates
HBM beside them (archive/profiles/r4g/step_breakdown_8b_full.txt).  Here the hand-written MFMA GEMM
(csrc/kernels/gemm8.hip, ``G8_EPI_ROPE`` / ``G8_EPI_SWIGLU``) applies them to its accumulators
before the stores, so neither the [T, 6144] qkv activation nor a separate SwiGLU pass ever
touches HBM:

  * ``qkv_attention``  x -> (q, k, v) rotated, head-major, straight from the GEMM -> flash
    attention; backward = attention backward -> inverse-RoPE merge -> dX / dW GEMMs.
  * ``gate_up_swiglu`` x -> (gu, m = silu(g) u) from ONE GEMM; gu is kept for the backward
    (SwiGLU backward -> dX / dW GEMMs).
  * ``gate_up_swiglu_down`` the same plus the down projection, so that its backward can run the
    down projection's dX GEMM with the SwiGLU backward in the epilogue (``G8_EPI_SWIGLU_BWD``):
    dgu straight from dy, W_down and the saved gu; the [T, F] dm never touches HBM and the
    separate swiglu_bwd pass (reads dm + gu, writes dgu) is gone.

The weight gradients go the ``_LinearFn`` way (written by the dW GEMM straight into the
owner's buffer).  Bitwise, each epilogue equals the GEMM followed by the kernel it replaces
(both round the product to bf16 first and then apply the same expression).
``MXLLM_FUSED_EPI=0`` restores the unfused ops (A/B).
"""
from __future__ import annotations

import math
import os

import torch

from . import gemm
from ._ext import native, use_native
from .linear import param_weight_grad

_ON = os.environ.get("MXLLM_FUSED_EPI", "1") != "0"
# the down projection's dX GEMM writes dgu through the SwiGLU backward epilogue (A/B: 0 = dm + swiglu_bwd)
_BWD_ON = os.environ.get("MXLLM_FUSED_SWIGLU_BWD", "1") != "0"


def _x2(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(-1, x.shape[-1])


def _norm_input(h: torch.Tensor, nw: torch.Tensor, eps: float) -> torch.Tensor:
    """x = rmsnorm(h) * nw recomputed (bitwise the forward's: the same kernel on the same h)."""
    return native().rmsnorm_fwd(h.reshape(-1, h.shape[-1]).contiguous(), None, nw, eps, 0)[0]


def _g8_operands_ok(a2: torch.Tensor, w: torch.Tensor) -> bool:
    """What ``mx_gemm8_epi`` (csrc/kernels/gemm8.hip) checks of two k-contiguous operands beyond the
    shapes: row strides in 16-B units, 16-B aligned bases, and both operand spans
    (256 rows of A, all N rows of W) under 2^31 bytes -- so a predicate that says yes never meets a
    declined launch (a 405B-class gate-up, 106,496 x 16,384, is over the span and stays unfused)."""
    lda, ldb = a2.stride(0), w.stride(0)
    return (lda % 8 == 0 and ldb % 8 == 0 and lda >= a2.shape[1] and ldb >= w.shape[1]
            and a2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and 256 * lda * 2 < 2 ** 31 and w.shape[0] * ldb * 2 < 2 ** 31)


def qkv_attention_ok(x: torch.Tensor, w: torch.Tensor, B: int, S: int, Hq: int, Hkv: int, D: int) -> bool:
    """Shapes the fused qkv epilogue takes (full fine-tuning: no LoRA buffer)."""
    x2 = _x2(x)
    return (_ON and use_native(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and D == 128
            and S % 256 == 0 and x2.shape[0] == B * S and x2.shape[1] % 64 == 0 and x2.stride(1) == 1
            and w.stride(1) == 1 and w.shape[0] == (Hq + 2 * Hkv) * D and not gemm.deterministic()
            and _g8_operands_ok(x2, w))


class _QKVAttentionFn(torch.autograd.Function):
    """o = attention(rope(split(x W^T))) with the projection, RoPE and head split in one GEMM.
    ``norm`` = (h, nw, eps): x = rmsnorm(h) nw is NOT saved but recomputed for dW."""

    @staticmethod
    def forward(ctx, x, w, cos, sin, B, S, Hq, Hkv, D, causal, out_pad, h, nw, eps):
        from .attention import _AttnBlockFn  # noqa: F401  (same kernels, same saved layout)

        ops = native()
        x2 = _x2(x)
        dev = x.device
        q = torch.empty(B, Hq, S, D, dtype=x.dtype, device=dev)
        k = torch.empty(B, Hkv, S, D, dtype=x.dtype, device=dev)
        v = torch.empty_like(k)
        if not ops.gemm8_rope(x2, w, cos, sin, B, S, Hq, Hkv, q, k, v):
            raise RuntimeError("gemm8_rope declined a shape qkv_attention_ok accepted")
        o, lse = ops.attn_fwd(q, k, v, causal, 1.0 / math.sqrt(D), out_pad)
        keep_x = h is None
        ctx.save_for_backward(x2 if keep_x else h, w, q, k, v, o, lse, cos, sin, nw)
        ctx.wp = w if w.is_leaf else None
        ctx.dims = (B, S, Hq, Hkv, D, causal, x.shape, keep_x, eps)
        return o.view(B * S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        from .attention import backward_dqkv

        xs, w, q, k, v, o, lse, cos, sin, nw = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, xshape, keep_x, eps = ctx.dims
        dqkv = backward_dqkv(do, q, k, v, o, lse, cos, sin, causal, 0)
        del q, k, v, o, lse
        dx = gemm.mm("nn", dqkv, w).view(xshape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = xs if keep_x else _norm_input(xs, nw, eps)
            dw = param_weight_grad(ctx.wp, dqkv, x2)
        return dx, dw, None, None, None, None, None, None, None, None, None, None, None, None


def qkv_attention(x: torch.Tensor, w: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, B: int, S: int,
                  Hq: int, Hkv: int, D: int, causal: bool = True, out_pad: int = 0,
                  norm: tuple | None = None) -> torch.Tensor:
    """[B*S, H] -> attention output [B*S, Hq*D] through the fused qkv epilogue (callers check
    ``qkv_attention_ok``).  ``norm`` = (h, nw, eps) when x = rmsnorm(h) nw should be recomputed
    in the backward instead of saved."""
    h, nw, eps = norm if norm is not None else (None, None, 0.0)
    return _QKVAttentionFn.apply(x, w, cos, sin, B, S, Hq, Hkv, D, causal, out_pad, h, nw, eps)


def gate_up_swiglu_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    x2 = _x2(x)
    return (_ON and use_native(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x2.shape[0] % 256 == 0 and x2.shape[1] % 64 == 0 and w.shape[0] % 256 == 0 and x2.stride(1) == 1
            and w.stride(1) == 1 and not gemm.deterministic() and _g8_operands_ok(x2, w))


class _GateUpSwiGLUFn(torch.autograd.Function):
    """m = silu(x Wg^T) * (x Wu^T) from ONE GEMM whose epilogue also writes gu for the backward."""

    @staticmethod
    def forward(ctx, x, w, out_pad, h, nw, eps):
        x2 = _x2(x)
        T, F2 = x2.shape[0], w.shape[0]
        gu = torch.empty(T, F2, dtype=x.dtype, device=x.device)
        mbuf = torch.empty(T, F2 // 2 + out_pad, dtype=x.dtype, device=x.device)
        m = mbuf[:, :F2 // 2]
        if not native().gemm8_swiglu(x2, w, gu, m):
            raise RuntimeError("gemm8_swiglu declined a shape gate_up_swiglu_ok accepted")
        keep_x = h is None
        ctx.save_for_backward(x2 if keep_x else h, w, gu, nw)
        ctx.wp = w if w.is_leaf else None
        ctx.dims = (x.shape, keep_x, eps)
        return m

    @staticmethod
    def backward(ctx, dm):
        xs, w, gu, nw = ctx.saved_tensors
        xshape, keep_x, eps = ctx.dims
        dgu = native().swiglu_bwd(dm.contiguous(), gu, 0)
        del gu
        dx = gemm.mm("nn", dgu, w).view(xshape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = xs if keep_x else _norm_input(xs, nw, eps)
            dw = param_weight_grad(ctx.wp, dgu, x2)
        return dx, dw, None, None, None, None


def gate_up_swiglu(x: torch.Tensor, w: torch.Tensor, out_pad: int = 0, norm: tuple | None = None) -> torch.Tensor:
    """m = swiglu(x W^T) [T, F] with W = [gate; up] (callers check ``gate_up_swiglu_ok``);
    ``out_pad``: the result is the left part of a [T, F + out_pad] buffer."""
    h, nw, eps = norm if norm is not None else (None, None, 0.0)
    return _GateUpSwiGLUFn.apply(x, w, out_pad, h, nw, eps)


def swiglu_bwd_gemm(dy: torch.Tensor, wd: torch.Tensor, gu: torch.Tensor, want_m: bool = False):
    """(dgu, m or None) = SwiGLU backward of dm = dy W_down from the saved gu, through the gemm8
    epilogue when it takes the shape, else the NN GEMM + swiglu_bwd(_m) pass (same bits where the
    GEMM dispatch picks gemm8 for dm: the epilogue's main loop is the plain kernel's)."""
    if _BWD_ON and use_native(dy) and not gemm.deterministic():
        dgu = torch.empty_like(gu)
        m = torch.empty(gu.shape[0], gu.shape[1] // 2, dtype=gu.dtype, device=gu.device) if want_m else None
        if native().gemm8_swiglu_bwd(dy, wd, gu, dgu, m):
            return dgu, m
    dm = gemm.mm("nn", dy, wd).contiguous()
    if want_m:
        return native().swiglu_bwd_m(dm, gu.contiguous())
    return native().swiglu_bwd(dm, gu, 0), None


def gate_up_swiglu_down_ok(x: torch.Tensor, wgu: torch.Tensor, wd: torch.Tensor) -> bool:
    return (_BWD_ON and gate_up_swiglu_ok(x, wgu) and wd.dim() == 2 and wd.dtype == torch.bfloat16
            and 2 * wd.shape[1] == wgu.shape[0] and wd.shape[1] % 256 == 0 and wd.shape[0] % 64 == 0
            and wd.stride(1) == 1 and wd.stride(0) % 8 == 0 and wd.data_ptr() % 16 == 0
            and 256 * wd.shape[0] * 2 < 2 ** 31 and wd.shape[0] * wd.stride(0) * 2 < 2 ** 31)


class _GateUpSwiGLUDownFn(torch.autograd.Function):
    """y = swiglu(x Wgu^T) Wd^T: the gate-up GEMM with the SwiGLU epilogue, then the down GEMM;
    backward: dgu from the down projection's dX GEMM epilogue, dWd from the saved m, then the
    gate-up dX / dW GEMMs.  Weight gradients go the ``_LinearFn`` way.

    ``recompute_m``: m is NOT saved (the activation-memory budget of the un-checkpointed layers of
    a selectively checkpointed run, models/llama.py ``_recompute_m``): the down projection's dX
    GEMM epilogue writes the recomputed m next to dgu (``G8_EPI_SWIGLU_BWD`` with ``ep.m``) for
    dWd -- the same saved tensors as the unfused recompute path (gu, and h when x is rebuilt), but
    no standalone SwiGLU pass in the forward."""

    @staticmethod
    def forward(ctx, x, wgu, wd, h, nw, eps, recompute_m=False):
        x2 = _x2(x)
        T, F2 = x2.shape[0], wgu.shape[0]
        gu = torch.empty(T, F2, dtype=x.dtype, device=x.device)
        m = torch.empty(T, F2 // 2, dtype=x.dtype, device=x.device)
        if not native().gemm8_swiglu(x2, wgu, gu, m):
            raise RuntimeError("gemm8_swiglu declined a shape gate_up_swiglu_down_ok accepted")
        y = gemm.mm("tn", m, wd)
        keep_x = h is None
        if recompute_m:
            del m
            m = None
        ctx.save_for_backward(x2 if keep_x else h, wgu, wd, gu, m, nw)
        ctx.wgp = wgu if wgu.is_leaf else None
        ctx.wdp = wd if wd.is_leaf else None
        ctx.dims = (x.shape, keep_x, eps, bool(recompute_m))
        return y.view(*x.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xs, wgu, wd, gu, m, nw = ctx.saved_tensors
        xshape, keep_x, eps, rec = ctx.dims
        dy2 = dy.reshape(-1, wd.shape[0])
        dgu, m_re = swiglu_bwd_gemm(dy2, wd, gu, want_m=rec and ctx.needs_input_grad[2])
        if rec:
            m = m_re
        del gu
        dwd = param_weight_grad(ctx.wdp, dy2, m) if ctx.needs_input_grad[2] else None
        del m
        dx = gemm.mm("nn", dgu, wgu).view(xshape) if ctx.needs_input_grad[0] else None
        dwgu = None
        if ctx.needs_input_grad[1]:
            x2 = xs if keep_x else _norm_input(xs, nw, eps)
            dwgu = param_weight_grad(ctx.wgp, dgu, x2)
        return dx, dwgu, dwd, None, None, None, None


def gate_up_swiglu_down(x: torch.Tensor, wgu: torch.Tensor, wd: torch.Tensor,
                        norm: tuple | None = None, recompute_m: bool = False) -> torch.Tensor:
    """The MLP body swiglu(x Wgu^T) Wd^T (callers check ``gate_up_swiglu_down_ok``); ``norm`` as in
    ``gate_up_swiglu``; ``recompute_m``: keep only gu, rebuild m in the backward's dm GEMM."""
    h, nw, eps = norm if norm is not None else (None, None, 0.0)
    return _GateUpSwiGLUDownFn.apply(x, wgu, wd, h, nw, eps, bool(recompute_m))
