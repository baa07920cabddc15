"""Linear layers: plain (hipBLASLt via torch.matmul) and fused multi-adapter LoRA.

A fused projection (Wqkv = [Wq; Wk; Wv], Wgu = [Wg; Wu]) carries one LoRA
adapter of rank r per output split.  All splits share the input, so
  * A is one [n*r, in] matrix: the down-projection t = x A^T is ONE skinny GEMM;
  * B is one BLOCK-DIAGONAL [N, n*r] matrix (split i's B_i in rows of split i,
    columns i*r..(i+1)*r; zeros elsewhere, never updated because their
    gradient is written as exact zeros): the up-projection is ONE GEMM.
Adapters are bf16 compute weights (fp32 master + Adam state live in the
flat optimizer buffers), so no per-call casts.

MI355X/hipBLASLt fusion: the LoRA term is not added with a separate
read-modify-write of the (huge) projection output.  It is written first and
then consumed as the C input of the base GEMM (beta = 1), whose epilogue reads
it while the GEMM is compute-bound (measured: beta=1 runs at the same
TFLOP/s as beta=0 on every Llama-3.1 projection shape):
  forward : y  = s t B^T            ; y  += x  W^T   (base GEMM, C = y)
  backward: g  = s dy B             ; dx  = g A      ; dx += dy W (base GEMM, C = dx)
            dB_i = s dy_i^T t_i (diagonal blocks only) ; dA = g^T x
Only x and the tiny t are saved for backward; the frozen base weight's
gradient is never formed.  The LoRA scale rides in the GEMM alpha, and when
the trainer has pre-attached flat .grad buffers the adapter gradients are
accumulated into them by the GEMMs themselves (beta = 1) — no zero-fill,
cast or accumulate kernels — and DDP is told via ``mark_ready``.
"""
from __future__ import annotations

import math
import os
from typing import Sequence

import torch
import torch.nn.functional as F

from ..parallel.grad_ready import direct_grad, direct_grad32, mark_ready
from . import gemm
from ._ext import native, use_native


class _LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, a, b, scaling, splits, r):
        x2 = x.reshape(-1, x.shape[-1])
        t = torch.matmul(x2, a.t())  # [T, n*r]
        y = torch.empty(x2.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        y.addmm_(t, b.t(), beta=0.0, alpha=scaling)  # LoRA term first (scale folded into alpha) ...
        y.addmm_(x2, w.t())  # ... then the base GEMM with C = y (beta = 1)
        ctx.save_for_backward(x2, w, a, b, t)
        ctx.scaling, ctx.splits, ctx.r, ctx.xshape = scaling, tuple(splits), r, x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, a, b, t = ctx.saved_tensors
        s, r = ctx.scaling, ctx.r
        dy2 = dy.reshape(-1, dy.shape[-1])
        g = torch.empty(dy2.shape[0], a.shape[0], dtype=dy2.dtype, device=dy2.device)
        g.addmm_(dy2, b, beta=0.0, alpha=s)  # [T, n*r] (block-diagonal B)
        # adapter grads: accumulate straight into the (flat) .grad buffers when
        # they exist (trainer-managed), otherwise hand them to autograd
        ga, gb = direct_grad(a) if ctx.needs_input_grad[2] else None, direct_grad(b) if ctx.needs_input_grad[3] else None
        da = db = None
        if ctx.needs_input_grad[2]:
            if ga is not None:
                ga.addmm_(g.t(), x2)
                mark_ready(a)
            else:
                da = torch.matmul(g.t(), x2)
        if ctx.needs_input_grad[3]:
            tgt = gb if gb is not None else torch.zeros_like(b)
            off = 0
            for i, n_i in enumerate(ctx.splits):
                tgt[off:off + n_i, i * r:(i + 1) * r].addmm_(dy2[:, off:off + n_i].t(), t[:, i * r:(i + 1) * r],
                                                            beta=1.0 if gb is not None else 0.0, alpha=s)
                off += n_i
            if gb is not None:
                mark_ready(b)
            else:
                db = tgt
        dx = torch.matmul(g, a)
        dx.addmm_(dy2, w)  # base dX GEMM with C = g A (beta = 1)
        return dx.view(ctx.xshape), None, da, db, None, None, None


def _padded_rows(t: torch.Tensor, pad: int) -> torch.Tensor | None:
    """If ``t`` [T, n] is the left part of a [T, n + pad] buffer (written that
    way by the producing kernel), return a view of the whole buffer that does
    NOT share ``t``'s autograd version counter (writing the pad columns must not
    invalidate tensors saved for backward that alias the left part)."""
    if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) != t.shape[1] + pad:
        return None
    st = t.untyped_storage()
    need = (t.storage_offset() + t.shape[0] * t.stride(0)) * t.element_size()
    if st.nbytes() < need:
        return None
    full = torch.empty(0, dtype=t.dtype, device=t.device)
    full.set_(st, t.storage_offset(), (t.shape[0], t.shape[1] + pad), (t.stride(0), 1))
    return full


def _augment(t: torch.Tensor, pad: int) -> torch.Tensor:
    full = _padded_rows(t, pad)
    if full is None:  # producer did not pad (e.g. CPU reference path): one copy
        full = torch.empty(t.shape[0], t.shape[1] + pad, dtype=t.dtype, device=t.device)
        full[:, :t.shape[1]].copy_(t)
    return full


_LORA_KERNELS = os.environ.get("MXLLM_LORA_KERNELS", "1") != "0"  # A/B switch (benchmarks)


def _lora_native(x2: torch.Tensor, N: int, K: int, splits, r: int, wbt) -> bool:
    """Shapes the hand-written LoRA kernels (csrc/kernels/lora.hip) take; others
    (tiny test models) use hipBLASLt for the rank-r products."""
    return (_LORA_KERNELS and wbt is not None and use_native(x2) and x2.shape[0] % 64 == 0 and K % 64 == 0 and r % 16 == 0
            and r <= 64 and all(n % 64 == 0 for n in splits) and x2.dtype == torch.bfloat16)


def _lora_aug_backward(ctx, xa, wbuf, dy, dy_tail: bool, need_a: bool, need_b: bool):
    """Backward of the augmented LoRA projection (``_LoRAAugFn``; also the LoRA half of
    ``_LoRAQKVAttnFn``): (dx reshaped to the input, dA or None, dB or None).  ``ctx`` carries
    ``dims`` = (N, K, s, splits, r, pad, xshape, nat, tr) and ``lora_a`` / ``lora_b`` / ``wbt`` / ``wxt``."""
    N, K, s, splits, r, pad, xshape, nat, tr = ctx.dims
    R = r * len(splits)
    dy2 = dy.reshape(-1, N)
    dya = _padded_rows(dy2, pad) if dy_tail else None
    if dya is None:  # ``dy_tail``: the SwiGLU backward already wrote s dy B into the pad columns
        dya = _augment(dy2, pad)
        if nat:
            native().lora_xwt(dy2, ctx.wbt, dya[:, N:], s, len(splits) * r)  # g = s dy B, zero in the pad columns
        else:
            bmat = wbuf[K:, :N].t() if tr else wbuf[:N, K:]  # B [N, pad]
            dya[:, N:].addmm_(dy2, bmat, beta=0.0, alpha=s)
    g = dya[:, N:N + R]
    x2, st = xa[:, :K], xa[:, K:K + R]
    da = db = None
    ga = direct_grad(ctx.lora_a) if need_a else None
    gb = direct_grad(ctx.lora_b) if need_b else None
    if nat and need_a and need_b:
        # dA and every diagonal dB_i in one launch, straight into the flat grads when present
        acc = ga is not None and gb is not None
        tga = ga if acc else torch.empty(R, K, dtype=dy2.dtype, device=dy2.device)
        tgb = gb if acc else torch.zeros(N, R, dtype=dy2.dtype, device=dy2.device)
        native().lora_grads(x2, dy2, dya[:, N:], xa[:, K:], tga, tgb, list(splits), r, acc)
        if acc:
            mark_ready(ctx.lora_a)
            mark_ready(ctx.lora_b)
        else:
            da, db = tga, tgb
    else:
        if need_a:
            if ga is not None:
                ga.addmm_(g.t(), x2)
                mark_ready(ctx.lora_a)
            else:
                da = torch.mm(g.t(), x2)
        if need_b:
            tgt = gb if gb is not None else torch.zeros(N, R, dtype=dy2.dtype, device=dy2.device)
            off = 0
            for i, n_i in enumerate(splits):
                tgt[off:off + n_i, i * r:(i + 1) * r].addmm_(dy2[:, off:off + n_i].t(), st[:, i * r:(i + 1) * r],
                                                            beta=1.0 if gb is not None else 0.0)
                off += n_i
            if gb is not None:
                mark_ready(ctx.lora_b)
            else:
                db = tgt
    if tr:  # [W; A]^T is the leading K rows of the transposed buffer: TN form
        dx = gemm.mm("tn", dya, wbuf[:K, :])
    elif ctx.wxt is not None:  # reduction-contiguous image of [W; A]: hipBLASLt "TN"
        dx = gemm.mm("tn", dya, ctx.wxt)
    else:  # the n-contiguous weight itself ("NN": gemm8 where it wins, csrc/kernels/gemm8.hip)
        dx = gemm.mm("nn", dya, wbuf[:, :K])
    return dx.view(xshape), da, db


class _LoRAAugFn(torch.autograd.Function):
    """LoRA projection as ONE augmented GEMM per direction (FusedLinear, models/llama.py).

    wbuf [N+Rp, K+Rp] = [[W, B], [A, 0]] (A / B zero-padded to Rp rows / cols;
    the adapter parameters ``a`` / ``b`` are autograd inputs, the GEMMs read
    their copies in wbuf, refreshed by the owner after every update):
      forward : x_aug  = [x | s x A^T]            (tail written in place)
                y      = x_aug @ wbuf[:N, :]^T    = x W^T + s (x A^T) B^T
      backward: dy_aug = [dy | s dy B]            (tail written in place)
                dx     = dy_aug @ wbuf[:, :K]     = dy W + (s dy B) A
                dA = (s dy B)^T x ;  dB_i = dy_i^T (s x A_i^T)  (diagonal blocks)
    The producers of x and dy (RMSNorm, SwiGLU, attention, RoPE-merge kernels)
    write them as the left part of [T, K+Rp] / [T, N+Rp] buffers, so the only
    extra traffic is the rank-Rp tail — no read-modify-write of the [T, N]
    output or the [T, K] input gradient (measured at the 70B shapes: qkv fwd
    0.79 -> 0.68 ms, gu fwd 2.66 -> 2.47 ms, down bwd 1.56 -> 1.47 ms).
    The rank-r products (the two tails, dA and every dB_i) run on the HIP
    kernels of csrc/kernels/lora.hip — one streaming pass over x or dy each,
    dA and all dB_i in ONE launch — with ``wbt`` = B^T as the k-contiguous
    operand of s dy B; hipBLASLt handles them for shapes those kernels do not take.
    """

    @staticmethod
    def forward(ctx, x, a, b, wbuf, scaling, splits, r, pad, wbt, wxt=None, wa=None, x_tail=False, dy_tail=False):
        tr = wa is not None  # transposed buffer [[W^T, A^T], [B^T, 0]] (FusedLinear ``transposed``)
        if tr:
            K, N = wbuf.shape[0] - pad, wbuf.shape[1] - pad
        else:
            N, K = wbuf.shape[0] - pad, wbuf.shape[1] - pad
        x2 = x.reshape(-1, K)
        nat = _lora_native(x2, N, K, splits, r, wbt)
        xa = _padded_rows(x2, pad) if x_tail else None
        if xa is None:  # ``x_tail``: the producer (SwiGLU) already wrote s x A^T into the pad columns
            xa = _augment(x2, pad)
            amat = wa if tr else wbuf[N:, :K]  # A rows [pad, K] (zero rows past n*r), k-contiguous
            if nat:
                native().lora_xwt(x2, amat, xa[:, K:], scaling, a.shape[0])  # s t, zero in the pad columns
            else:
                xa[:, K:].addmm_(x2, amat.t(), beta=0.0, alpha=scaling)
        y = gemm.mm("nn", xa, wbuf[:, :N]) if tr else gemm.mm("tn", xa, wbuf[:N, :])
        ctx.save_for_backward(xa, wbuf)
        ctx.lora_a, ctx.lora_b, ctx.wbt, ctx.wxt = a, b, wbt, wxt
        ctx.dims = (N, K, scaling, tuple(splits), r, pad, x.shape, nat, tr)
        ctx.dy_tail = dy_tail
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        xa, wbuf = ctx.saved_tensors
        dx, da, db = _lora_aug_backward(ctx, xa, wbuf, dy, ctx.dy_tail, ctx.needs_input_grad[1],
                                        ctx.needs_input_grad[2])
        return dx, da, db, None, None, None, None, None, None, None, None, None, None


def lora_linear_aug(x: torch.Tensor, a: torch.Tensor, b: torch.Tensor, wbuf: torch.Tensor, splits: Sequence[int],
                    scaling: float, pad: int, wbt: torch.Tensor | None = None,
                    wxt: torch.Tensor | None = None, wa: torch.Tensor | None = None,
                    x_tail: bool = False, dy_tail: bool = False) -> torch.Tensor:
    """LoRA projection through the augmented weight buffer (see _LoRAAugFn);
    ``wxt``: optional [K, N+pad] transposed image of wbuf[:, :K] for dX;
    ``wa``: given for a TRANSPOSED buffer [[W^T, A^T], [B^T, 0]] (A rows, k-contiguous);
    ``x_tail`` / ``dy_tail``: the producer of x (forward) / of the output gradient (backward)
    writes the rank-r tail itself (mxllm/ops/activation.py fused SwiGLU); used whenever the
    tensor arrives in its padded buffer, recomputed otherwise."""
    r = a.shape[0] // len(splits)
    return _LoRAAugFn.apply(x, a, b, wbuf, scaling, tuple(splits), r, pad, wbt, wxt, wa, bool(x_tail), bool(dy_tail))


_LORA_QKV_ROPE = os.environ.get("MXLLM_LORA_QKV_ROPE", "1") != "0"  # A/B switch


def lora_qkv_attention_at(x: torch.Tensor, lin, B: int, S: int, Hq: int, Hkv: int, D: int) -> int:
    """The tail-balanced split column ``at`` (> 0) when the LoRA q/k/v projection ``lin`` (a FusedLinear
    with an augmented, non-transposed buffer) can run as ``lora_qkv_attention``: exactly when its
    unfused forward GEMM would run the tail-balanced gemm8 launch (the dispatch table's ``tail``
    entry for the augmented shape), whose RoPE variant then replaces GEMM + rope_split; 0 otherwise."""
    from .fused import _g8_operands_ok

    if not (_LORA_QKV_ROPE and lin.lora_r > 0 and lin.augmented() and not lin.transposed and D == 128
            and S % 256 == 0 and use_native(x) and x.dtype == torch.bfloat16 and not gemm.deterministic()):
        return 0
    N, K, pad = sum(lin.splits), lin.in_features, lin.pad
    x2 = x.reshape(-1, x.shape[-1])
    if N != (Hq + 2 * Hkv) * D or x2.shape[0] != B * S or x2.shape[1] != K:
        return 0
    xa = _padded_rows(x2, pad)
    if xa is None or not _g8_operands_ok(xa, lin.wbuf[:N, :]):
        return 0
    key = ("tn", B * S, N, K + pad, "bf16")
    if not gemm.schedule("tn", B * S, N, K + pad, torch.bfloat16):
        return 0
    gemm._table()
    at = gemm._TAIL.get(key, 0)
    return at if at > 0 else 0


def _lora_aug_input(x2, a, wbuf, amat, scaling, N, K, pad, nat):
    """x_aug = [x | s x A^T] in x's padded row buffer (see _LoRAAugFn)."""
    xa = _augment(x2, pad)
    if nat:
        native().lora_xwt(x2, amat, xa[:, K:], scaling, a.shape[0])  # s t, zero in the pad columns
    else:
        xa[:, K:].addmm_(x2, amat.t(), beta=0.0, alpha=scaling)
    return xa


class _LoRAQKVAttnFn(torch.autograd.Function):
    """LoRA q/k/v projection + RoPE + head split + flash attention in one autograd node.  The augmented
    GEMM of ``_LoRAAugFn`` runs as the tail-balanced gemm8 launch with the RoPE epilogue
    (csrc/kernels/gemm8.hip ``mx_gemm8_rope_tail``: q / k / v written head-major by the plain part's
    epilogue and by the split part's sum pass), so neither the [T, N] qkv activation nor the
    rope_split pass touches HBM -- bitwise the GEMM + rope_split it replaces.  Backward: the attention
    backward writes d(qkv) (inverse RoPE applied) into a buffer padded for the LoRA tail, then the
    LoRA backward of ``_LoRAAugFn``."""

    @staticmethod
    def forward(ctx, x, a, b, wbuf, scaling, splits, r, pad, wbt, wxt, cos, sin, B, S, Hq, Hkv, D, causal, out_pad,
                at):
        N, K = wbuf.shape[0] - pad, wbuf.shape[1] - pad
        x2 = x.reshape(-1, K)
        nat = _lora_native(x2, N, K, splits, r, wbt)
        xa = _lora_aug_input(x2, a, wbuf, wbuf[N:, :K], scaling, N, K, pad, nat)
        ops = native()
        q = torch.empty(B, Hq, S, D, dtype=x.dtype, device=x.device)
        k = torch.empty(B, Hkv, S, D, dtype=x.dtype, device=x.device)
        v = torch.empty_like(k)
        if not ops.gemm8_rope_tail(xa, wbuf[:N, :], cos, sin, B, S, Hq, Hkv, q, k, v, at):
            q, k, v = ops.rope_split(gemm.mm("tn", xa, wbuf[:N, :]), cos, sin, B, S, Hq, Hkv, D)
        o, lse = ops.attn_fwd(q, k, v, causal, 1.0 / math.sqrt(D), out_pad)
        ctx.save_for_backward(xa, wbuf, q, k, v, o, lse, cos, sin)
        ctx.lora_a, ctx.lora_b, ctx.wbt, ctx.wxt = a, b, wbt, wxt
        ctx.dims = (N, K, scaling, tuple(splits), r, pad, x.shape, nat, False)
        ctx.causal = causal
        return o.view(B * S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        from .attention import backward_dqkv

        xa, wbuf, q, k, v, o, lse, cos, sin = ctx.saved_tensors
        pad = ctx.dims[5]
        dqkv = backward_dqkv(do, q, k, v, o, lse, cos, sin, ctx.causal, pad)  # left part of [T, N + pad]
        del q, k, v, o, lse
        dx, da, db = _lora_aug_backward(ctx, xa, wbuf, dqkv, False, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return (dx, da, db) + (None,) * 17


def lora_qkv_attention(x: torch.Tensor, lin, cos: torch.Tensor, sin: torch.Tensor, B: int, S: int, Hq: int,
                       Hkv: int, D: int, at: int, causal: bool = True, out_pad: int = 0) -> torch.Tensor:
    """attention(rope(split(lora_qkv(x)))) -> [B*S, Hq*D] for the LoRA FusedLinear ``lin`` (callers take
    ``at`` from ``lora_qkv_attention_at``)."""
    r = lin.lora_a.shape[0] // len(lin.splits)
    return _LoRAQKVAttnFn.apply(x, lin.lora_a, lin.lora_b, lin.wbuf, lin.scaling, tuple(lin.splits), r, lin.pad,
                                lin.wbt, getattr(lin, "wxt", None), cos, sin, B, S, Hq, Hkv, D, causal, out_pad, at)


def transpose2d(t: torch.Tensor, scale: torch.Tensor | None = None) -> torch.Tensor:
    """Contiguous ``t.T`` of a 2-D row-major (row-strided) 16-bit tensor: the
    LDS-tiled HIP transpose on GPU (csrc/kernels/misc.hip), torch on CPU.
    ``scale``: optional 1-element f32 device tensor multiplied in (bf16 ``t``)."""
    if use_native(t):
        if t.stride(-1) != 1:
            t = t.contiguous()
        return native().transpose2d(t, scale)
    out = t.t().contiguous()
    return out if scale is None else (out * scale.to(out.dtype))


def copy2d_plan(pairs) -> tuple[list[list[int]], int]:
    """Descriptor rows and the block count of ONE ``copy2d_batched`` launch over ``pairs`` of 2-D
    16-bit (src, dst) views of equal shape (csrc/kernels/misc.hip): 4,096 elements per block, or
    one 64 x 64 source tile per block where the copy transposes (source rows contiguous, the
    destination a column-major view)."""
    rows, total = [], 0
    for s, d in pairs:
        assert s.shape == d.shape and s.dim() == 2 and s.element_size() == 2 and d.element_size() == 2
        r, c = s.shape
        rows.append([s.data_ptr(), d.data_ptr(), r, c, s.stride(0), d.stride(0), total, s.stride(1), d.stride(1)])
        if s.stride(1) == 1 and d.stride(0) == 1 and d.stride(1) != 1:
            total += ((r + 63) // 64) * ((c + 63) // 64)
        else:
            total += (r * c + 4095) // 4096
    return rows, total


_DW_TN = os.environ.get("MXLLM_DW_TN", "1") != "0"


def weight_grad_(out: torch.Tensor | None, dy: torch.Tensor, x: torch.Tensor, beta: float = 1.0,
                 dy_scale: torch.Tensor | None = None) -> torch.Tensor:
    """dW = dy^T x (reduction over the token dimension), accumulated into
    ``out`` (``out = beta * out + dW``; beta 0 ignores whatever ``out`` held)
    when given.

    Both activations are token-major, so the direct GEMM is hipBLASLt's
    reduction-strided "NT" kernel family (~0.93-1.15 PF on the Llama-3.1
    projections).  On GPU the two operands are first transposed into
    token-contiguous images by the HIP transpose (4.4-6.4 TB/s) and the GEMM
    runs in the reduction-contiguous form the forward uses: dW = dyT @ xT^T,
    12-20 % faster including the transposes
    (bench/dw_layout_probe.py, archive/profiles/r1e_dw_layout_probe.md).
    ``dy_scale``: 1-element device tensor multiplying dy (folded into dy's
    transpose on that path; the cross-entropy's upstream gradient)."""
    f32 = out is not None and out.dtype == torch.float32 and dy.dtype != torch.float32
    if use_native(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
        # token-major operands straight into the 8-phase MFMA GEMM (no transposes) where it wins
        odt = out.dtype if out is not None else dy.dtype
        if gemm.want("tt", dy.shape[1], x.shape[1], dy.shape[0], odt):
            sc = None if dy_scale is None else dy_scale.reshape(1).float()
            return gemm.mm("tt", dy, x, out=out, beta=beta if out is not None else 0.0, alpha_t=sc,
                           out_dtype=odt)
    if _DW_TN and use_native(dy) and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
        xt = transpose2d(x)
        dyt = transpose2d(dy, None if dy_scale is None else dy_scale.reshape(1).float())
        if out is None:
            return torch.mm(dyt, xt.t())
        if f32:  # bf16 operands, fp32 accumulate-into output (hipBLASLt D = C in fp32)
            return torch.ops.aten.addmm.dtype_out(out, dyt, xt.t(), torch.float32, beta=beta, out=out)
        return out.addmm_(dyt, xt.t(), beta=beta)
    if dy_scale is not None:
        dy = dy * dy_scale.to(dy.dtype)
    if out is None:
        return torch.mm(dy.t(), x)
    if f32:
        if dy.is_cuda:
            return torch.ops.aten.addmm.dtype_out(out, dy.t(), x, torch.float32, beta=beta, out=out)
        return out.addmm_(dy.t().float(), x.float(), beta=beta)
    return out.addmm_(dy.t(), x, beta=beta)


def param_weight_grad(wp: torch.Tensor | None, dy: torch.Tensor, x: torch.Tensor,
                      dy_scale: torch.Tensor | None = None) -> torch.Tensor | None:
    """Weight gradient of parameter ``wp`` for a backward pass.

    When an owner pre-attached ``wp.grad`` (the trainer's flat grad buffer, or a
    ZeRO-3 unit's gathered-gradient buffer) — or an fp32 target ``wp._mx_grad32``
    (fp32 gradient accumulation) — the dW GEMM writes straight into it —
    accumulating (beta 1), or overwriting (beta 0) when the owner flagged the
    buffer ``_mx_grad_fresh`` so it need not be zero-filled first — the owner is
    notified via ``mark_ready`` and None is returned.  Otherwise the dW tensor
    is returned for autograd to accumulate."""
    g = direct_grad(wp) if wp is not None else None
    if g is None and wp is not None:
        g = direct_grad32(wp)  # fp32 gradient accumulation: the GEMM writes fp32
    if g is None:
        return weight_grad_(None, dy, x, dy_scale=dy_scale)
    fresh = getattr(wp, "_mx_grad_fresh", False)
    # the trainer's fused clip norm (mxllm/train/trainer.py): a first write (beta 0) of a gradient
    # whose owner armed `_mx_sq` also leaves the per-tile sums of squares of the stored values
    armed = getattr(wp, "_mx_sq_done", None)
    sq = getattr(wp, "_mx_sq", None) if fresh and armed is False else None
    if sq is not None and g.dtype == dy.dtype == x.dtype == torch.bfloat16 and gemm.mm_sq(
            "tt", dy, x, g, sq, None if dy_scale is None else dy_scale.reshape(1).float()):
        wp._mx_sq_done = True
    else:
        if armed is True:  # a second write onto partials already taken: the trainer re-reads instead
            wp._mx_sq_done = "dirty"
        weight_grad_(g, dy, x, beta=0.0 if fresh else 1.0, dy_scale=dy_scale)
    if fresh:
        wp._mx_grad_fresh = False
    mark_ready(wp)
    return None


class _LinearFn(torch.autograd.Function):
    """y = x W^T whose weight gradient is accumulated by the dW GEMM itself into
    the preallocated flat .grad (beta = 1) — no separate dW tensor and no
    AccumulateGrad add pass over it (full fine-tuning: ~16 GB of weight
    gradient per 8B step) — and DDP is told via ``mark_ready``."""

    @staticmethod
    def forward(ctx, x, w):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, w)
        # the Parameter itself (its .grad is the direct-accumulation target): under
        # ZeRO-3 the saved ``w`` unpacks as a view of the re-gathered unit, not the leaf
        ctx.wp = w if w.is_leaf else None
        ctx.xshape = x.shape
        return gemm.mm("tn", x2, w).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        dx = gemm.mm("nn", dy2, w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = param_weight_grad(ctx.wp, dy2, x2) if ctx.needs_input_grad[1] else None
        return dx, dw


def _swiglu_nograd(gu: torch.Tensor) -> torch.Tensor:
    if use_native(gu):
        return native().swiglu_fwd(gu.contiguous(), 0)
    from . import reference as ref

    return ref.swiglu(gu)


class _SwiGLULinearFn(torch.autograd.Function):
    """y = swiglu(gu) W^T that keeps only ``gu`` for the backward and recomputes m = swiglu(gu)
    there (one elementwise pass) instead of saving it: m is the [T, F] activation of every MLP
    (70B, 8,192 tokens: 470 MB per layer), so memory-bound runs (selective activation
    checkpointing, config 4) keep more layers un-checkpointed for the same HBM.  The weight
    gradient goes the _LinearFn way (direct accumulation into the owner's buffer)."""

    @staticmethod
    def forward(ctx, gu, w):
        g2 = gu.reshape(-1, gu.shape[-1])
        m = _swiglu_nograd(g2)
        ctx.save_for_backward(g2, w)
        ctx.wp = w if w.is_leaf else None
        ctx.gshape = gu.shape
        return gemm.mm("tn", m, w).view(*gu.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        g2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        dgu = dw = None
        if use_native(g2):
            # dgu AND the recomputed m for dW from one pass over gu: the dX GEMM's SwiGLU-backward
            # epilogue (mxllm/ops/fused.py), else dm first and one swiglu_bwd_m pass over (dm, gu)
            from .fused import swiglu_bwd_gemm

            dgu, m = swiglu_bwd_gemm(dy2, w, g2, want_m=True)
            if ctx.needs_input_grad[1]:
                dw = param_weight_grad(ctx.wp, dy2, m)
            del m
        else:
            from . import reference as ref

            with torch.enable_grad():
                gr = g2.detach().requires_grad_(True)
                m = ref.swiglu(gr)
            if ctx.needs_input_grad[1]:
                dw = param_weight_grad(ctx.wp, dy2, m.detach())
            if ctx.needs_input_grad[0]:
                (dgu,) = torch.autograd.grad(m, gr, gemm.mm("nn", dy2, w))
        if dgu is not None and ctx.needs_input_grad[0]:
            dgu = dgu.view(ctx.gshape)
        else:
            dgu = None
        return dgu, dw


def swiglu_linear(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Training: ``linear(swiglu(gu), w)`` with m recomputed in the backward (_SwiGLULinearFn)."""
    return _SwiGLULinearFn.apply(gu, w)


class _NormedLinearFn(torch.autograd.Function):
    """y = x W^T for x = rmsnorm(h) * nw that does not save x: the backward recomputes it from the
    residual h the norm node keeps anyway (bitwise: csrc/kernels/rmsnorm.hip normalises the stored
    bf16 h in both variants), one [T, H] pass instead of a saved [T, H] activation per projection
    (70B, 8,192 tokens: 134 MB each for the qkv and gate-up inputs of every layer)."""

    @staticmethod
    def forward(ctx, x, h, nw, eps, w):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(h, nw, w)
        ctx.wp = w if w.is_leaf else None
        ctx.eps, ctx.xshape = eps, x.shape
        return gemm.mm("tn", x2, w).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        h, nw, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0])
        dx = gemm.mm("nn", dy2, w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[4]:
            h2 = h.reshape(-1, h.shape[-1])
            if use_native(h2):
                x2 = native().rmsnorm_fwd(h2.contiguous(), None, nw, ctx.eps, 0)[0]
            else:
                from . import reference as ref

                x2 = ref.rms_norm(h2, nw, ctx.eps)
            dw = param_weight_grad(ctx.wp, dy2, x2)
            del x2
        return dx, None, None, None, dw


def normed_linear(x: torch.Tensor, h: torch.Tensor, nw: torch.Tensor, eps: float, w: torch.Tensor) -> torch.Tensor:
    """Training: ``linear(x, w)`` where x = rms_norm(h, nw, eps), x recomputed in the backward
    (_NormedLinearFn)."""
    return _NormedLinearFn.apply(x, h, nw, eps, w)


# decode-sized GEMMs (bf16, no autograd) on the weight-streaming HIP kernel
# (csrc/kernels/skinny_gemm.hip) where it beat hipBLASLt inside the decode step
# (bench/serve_bench.py A/B, archive/profiles/r2x_skinny_gemm.md): one token row for every projection
# and the LM head; 2..SKINNY_M rows for weights of <= 128 M elements (all Llama-3.1-8B
# projections; the 70B ones lost at 4 rows).  MXLLM_SKINNY_M=0 keeps every GEMM on hipBLASLt.
SKINNY_M = int(os.environ.get("MXLLM_SKINNY_M", "8"))
_SKINNY_SMALL_W = 128 << 20


def _skinny_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    K, M = x2.shape[1], x2.shape[0]
    if M > 1 and w.shape[0] * K > _SKINNY_SMALL_W:
        return False
    return (M <= SKINNY_M and x2.is_cuda and x2.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and K % 512 == 0 and w.shape[0] % 16 == 0 and x2.stride(1) == 1
            and x2.stride(0) % 8 == 0 and w.stride(1) == 1 and w.stride(0) % 8 == 0 and use_native(x2))


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if w.requires_grad and torch.is_grad_enabled():
        return _LinearFn.apply(x, w)
    if SKINNY_M > 0 and x.shape[-1] == w.shape[1] and x.numel() // max(x.shape[-1], 1) <= SKINNY_M:
        x2 = x.reshape(-1, x.shape[-1])
        if x2.shape[0] > 0 and _skinny_ok(x2, w):
            return native().skinny_linear(x2, w).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w)


def linear_swiglu(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor | None:
    """Inference: ``swiglu(linear(x, w))`` for decode-sized row counts as ONE launch, with
    ``w = [gate; up]`` [2F, K] (csrc/kernels/skinny_gemm.hip SWO variant: the SwiGLU in
    the GEMM epilogue, bit-identical to the GEMM + SwiGLU kernels).  None when the fused
    kernel does not take the call (the caller then runs the two ops)."""
    if SKINNY_M <= 0 or x.dim() != 2 or (w.requires_grad and torch.is_grad_enabled()):
        return None
    if x.shape[1] != w.shape[1] or w.shape[0] % 16 or not 0 < x.shape[0] <= SKINNY_M:
        return None
    if not _skinny_ok(x, w):
        return None
    return native().skinny_linear_swiglu(x, w)


# rows up to which the RMSNorm runs in the decode GEMM's prologue (every workgroup recomputes the
# rows): measured same box, 8B decode batch 1 3.607 -> 3.479 ms and 70B 26.22 -> 24.98 ms, but batch 4
# 3.83 -> 4.04 ms (archive/profiles/r2s3_decode_ab/); the kernel takes up to 4
NORM_M = int(os.environ.get("MXLLM_NORM_FUSED_M", "2"))


def qkv_rope_ok(h: torch.Tensor, w: torch.Tensor, cos, sin, k_cache, v_cache, Hq: int, Hkv: int,
                norm: bool) -> bool:
    """Whether :func:`qkv_rope_linear` takes these shapes (``norm``: with the RMSNorm prologue)."""
    if SKINNY_M <= 0 or h.dim() != 2 or (w.requires_grad and torch.is_grad_enabled()):
        return False
    M, K = h.shape
    if not 0 < M <= (min(NORM_M, SKINNY_M) if norm else SKINNY_M) or (norm and M * K > 32768):
        return False
    if w.shape != ((Hq + 2 * Hkv) * 128, K) or k_cache.shape[-1] != 128 or k_cache.dtype != torch.bfloat16:
        return False
    return bool(_skinny_ok(h, w) and cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()
                and k_cache.is_contiguous() and v_cache.is_contiguous())


def qkv_rope_linear(delta, h: torch.Tensor, gamma, eps: float, w: torch.Tensor, cos, sin, pos, slots, k_cache,
                    v_cache, Hq: int, Hkv: int, block_table=None):
    """Inference, decode rows: the QKV projection with RoPE and the KV-cache append in the GEMM
    epilogue (csrc/kernels/skinny_gemm.hip ROPE) and, for 1-NORM_M rows, the (residual-add +)
    RMSNorm in its prologue; ``gamma`` None: ``h`` is already normalised; ``block_table``:
    paged caches (mxllm/serve/kvcache.py).  Returns
    (q [M, Hq, 128] rotated, new residual) or None when the fused kernel does not take the call."""
    if not qkv_rope_ok(h, w, cos, sin, k_cache, v_cache, Hq, Hkv, gamma is not None):
        return None
    norm = gamma is not None
    if norm and (gamma.dtype != torch.bfloat16 or not gamma.is_contiguous()):
        return None
    if delta is not None and (not norm or delta.shape != h.shape or delta.stride(1) != 1 or delta.stride(0) % 8):
        return None
    return native().skinny_qkv_rope(h, delta, gamma, float(eps), w, cos, sin, pos, slots, k_cache, v_cache, Hq, Hkv,
                                    block_table)


def norm_linear(delta: torch.Tensor | None, h: torch.Tensor, gamma: torch.Tensor, eps: float, w: torch.Tensor,
                swiglu: bool = False):
    """Inference, decode rows: ``(linear(rmsnorm(h + delta) * gamma, w), h + delta)`` as ONE
    launch (csrc/kernels/skinny_gemm.hip NORM: the RMSNorm in the GEMM prologue, same bits as
    the RMSNorm kernel + decode GEMM); with ``swiglu`` w = [gate; up] and the first output is
    silu(g) * u.  ``delta`` None: plain RMSNorm, the residual is ``h``.  None when the fused
    kernel does not take the call."""
    if SKINNY_M <= 0 or h.dim() != 2 or (w.requires_grad and torch.is_grad_enabled()):
        return None
    M, K = h.shape
    if not 0 < M <= min(NORM_M, SKINNY_M) or M * K > 32768 or h.stride(1) != 1 or w.shape[1] != K or w.shape[0] % 16:
        return None
    if gamma.dtype != torch.bfloat16 or not gamma.is_contiguous() or not _skinny_ok(h, w):
        return None
    if delta is not None and (delta.shape != h.shape or delta.dtype != h.dtype or delta.stride(1) != 1
                              or delta.stride(0) % 8):
        return None
    return native().skinny_norm_linear(h, delta, gamma, float(eps), w, bool(swiglu))


def lora_linear(x: torch.Tensor, w: torch.Tensor, a: torch.Tensor, b: torch.Tensor, splits: Sequence[int],
                scaling: float) -> torch.Tensor:
    """y = x W^T + scaling * (x A^T) Bbd^T with block-diagonal Bbd (see module doc)."""
    r = a.shape[0] // len(splits)
    return _LoRALinearFn.apply(x, w, a, b, scaling, tuple(splits), r)
