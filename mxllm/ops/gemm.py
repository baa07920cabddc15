"""GEMM dispatch between the hand-written 8-phase MFMA kernel (csrc/kernels/gemm8.hip) and
hipBLASLt / rocBLAS (``torch.mm`` with the tuned solution table, mxllm/utils/gemm_tuning.py).

Every training GEMM of a Llama step is one of four operand orders over row-major bf16 storage:

  form  A stored   B stored   computes          used for
  tn    [M][K]     [N][K]     A @ B^T           forward  y = x W^T
  nn    [M][K]     [K][N]     A @ B             input gradient  dX = dY W
  tt    [K][M]     [K][N]     A^T @ B           weight gradient dW = dY^T X (token-major operands)
  nt    [K][M]     [N][K]     A^T @ B^T         (unused; for completeness)

``gemm8`` is selected per (form, M, N, K, output dtype) only where it was measured faster
(entries with ``tail``: the tail-balanced launch, ``mx_gemm8_tail`` -- a last wave of at most half
the CUs runs as twice as many half-K workgroups, e.g. the 16 x 40-tile 70B qkv forward)
(``mxllm/tuning/gemm8_gfx950.json``, written from ``bench/gemm8_probe.py`` runs), or for every
shape it takes in deterministic mode (``MXLLM_DETERMINISTIC=1``: one workgroup per output tile,
a fixed K order, no split-K or atomics — the step is bitwise reproducible; vendor stream-K
solutions are not, archive/profiles/r3aa).  ``MXLLM_GEMM8=0`` disables it, ``=all`` forces it wherever
it takes the shape (A/B runs).
"""
from __future__ import annotations

import json
import os

import torch

from ._ext import native, use_native

_TABLE_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                           "gemm8_gfx950.json")
_TABLE: dict | None = None


def deterministic() -> bool:
    return os.environ.get("MXLLM_DETERMINISTIC", "0") == "1"


_TAIL: dict = {}


def _table() -> dict:
    global _TABLE
    if _TABLE is None:
        _TABLE = {}
        try:
            with open(_TABLE_PATH) as f:
                for e in json.load(f).get("wins", []):
                    key = (e["form"], e["M"], e["N"], e["K"], e["out"])
                    _TABLE[key] = int(e.get("ph", 8))
                    if e.get("tail"):
                        _TAIL[key] = int(e["tail"])
        except (OSError, ValueError, KeyError):
            pass
    return _TABLE


CUS = 256  # MI355X compute units: one gemm8 workgroup (256 x 256 tile) per CU at a time


def tail_split(M: int, N: int, K: int) -> int:
    """Split of the tail-balanced launch (mx_gemm8_tail), 0 if it does not apply: the tile grid leaves
    a last wave of at most half the CUs.  > 0: split at that COLUMN (whole waves of tiles in columns
    [0, N1)); < 0: split at ROW -value (when no column split gives whole waves)."""
    if M % 256 or N % 256 or K < 128:
        return 0
    nM, nN = M // 256, N // 256
    r = (nM * nN) % CUS
    if r == 0 or r > CUS // 2:
        return 0
    full = nM * nN - r
    if full % nM == 0 and 0 < full // nM < nN:
        return full // nM * 256
    if full % nN == 0 and 0 < full // nN < nM:
        return -(full // nN * 256)
    return 0


def _multi_rank() -> bool:
    """True in a process group of more than one rank.  The persistent gemm8 (table ``ph`` 5) gives
    each of its one-per-CU workgroups a FIXED share of the tiles; a collective kernel that holds CUs
    for its whole duration (RCCL's channels, the peer collectives) then delays the workgroups that
    cannot start, and with them the whole GEMM -- under ZeRO-3's reduce-scatters overlapped with the
    dW GEMMs that costs far more than the persistence wins (0.7 % of the world-1 config-4 proxy,
    profiles/r5e).  The one-tile-per-workgroup launch lets the hardware rebalance around them."""
    import torch.distributed as dist

    # asked only for ph-5 shapes (a few fp32 dW GEMMs per layer): not cached, so a process that
    # brings a group up or down later is still answered right
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _policy() -> str:
    return os.environ.get("MXLLM_GEMM8", "table")


def takes(form: str, M: int, N: int, K: int) -> bool:
    """Shape constraints of the kernel (mirrors mx_gemm8)."""
    if M % 256 or N % 256 or K <= 0:
        return False
    return K % 64 == 0 or form == "tt"


def schedule(form: str, M: int, N: int, K: int, out_dtype: torch.dtype) -> int:
    """0 = not on gemm8; else its phase schedule (8 or 4) for this shape."""
    pol = _policy()
    if pol == "0" or not takes(form, M, N, K):
        return 0
    ph = _table().get((form, M, N, K, "f32" if out_dtype == torch.float32 else "bf16"), 0)
    if ph == 5 and _multi_rank():
        ph = 4  # persistent kernel: world 1 only (see _multi_rank)
    if ph:
        return ph
    return DEFAULT_PH if (pol == "all" or deterministic()) else 0


DEFAULT_PH = int(os.environ.get("MXLLM_GEMM8_DEFAULT_PH", "4"))


def want(form: str, M: int, N: int, K: int, out_dtype: torch.dtype) -> bool:
    return schedule(form, M, N, K, out_dtype) > 0


# (A k-contiguous, B k-contiguous) per form
_KC = {"tn": (True, True), "nn": (True, False), "tt": (False, False), "nt": (False, True)}


def _dims(form, a, b):
    if form == "tn":
        return a.shape[0], b.shape[0], a.shape[1]
    if form == "nn":
        return a.shape[0], b.shape[1], a.shape[1]
    if form == "tt":
        return a.shape[1], b.shape[1], a.shape[0]
    return a.shape[1], b.shape[0], a.shape[0]


def mm(form: str, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, beta: float = 0.0,
       alpha_t: torch.Tensor | None = None, out_dtype: torch.dtype | None = None) -> torch.Tensor:
    """``out = beta * out + alpha_t * op(a) op(b)`` in operand order ``form`` (module doc).
    ``out`` None: a new [M, N] tensor of ``out_dtype`` (default: a's dtype) and beta is 0.
    ``alpha_t``: optional 1-element f32 device scalar (no host sync)."""
    M, N, K = _dims(form, a, b)
    odt = out.dtype if out is not None else (out_dtype or a.dtype)
    if out is None:
        out = torch.empty(M, N, dtype=odt, device=a.device)
        beta = 0.0
    ph = (schedule(form, M, N, K, odt) if use_native(a) and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
          and odt in (torch.bfloat16, torch.float32) else 0)
    if ph:
        a_kc, b_kc = _KC[form]
        t = _TAIL.get((form, M, N, K, "f32" if odt == torch.float32 else "bf16"), 0)
        if (t and beta == 0.0 and alpha_t is None and odt == torch.bfloat16
                and native().gemm8_tail(a, a_kc, b, b_kc, out, abs(t), t < 0, ph)):
            return out
        if native().gemm8(a, a_kc, b, b_kc, out, float(beta), alpha_t, 1.0, ph):
            return out
    A = a if form in ("tn", "nn") else a.t()
    B = b.t() if form in ("tn", "nt") else b
    if alpha_t is not None:
        A = A * alpha_t.to(A.dtype)
    if odt == a.dtype:
        if beta == 0.0:
            return torch.mm(A, B, out=out)
        return out.addmm_(A, B, beta=beta)
    if a.is_cuda:  # bf16 operands, fp32 output (hipBLASLt D = C in fp32)
        return torch.ops.aten.addmm.dtype_out(out, A, B, odt, beta=beta, out=out)
    return out.mul_(beta).add_(A.float() @ B.float()) if beta != 0.0 else out.copy_(A.float() @ B.float())


def mm_sq(form: str, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, sq: torch.Tensor,
          alpha_t: torch.Tensor | None = None) -> bool:
    """``out = alpha_t * op(a) op(b)`` (bf16, beta 0) on gemm8 that also writes one fp32 sum of squares of
    the stored values per 256 x 256 output tile into ``sq`` (row-major tile order).  Only where the
    dispatch puts this shape on the plain 4-phase gemm8 anyway (same kernel, same bits in ``out``);
    False: nothing launched, the caller takes ``mm``."""
    M, N, K = _dims(form, a, b)
    if not (use_native(a) and a.dtype == b.dtype == out.dtype == torch.bfloat16 and M % 256 == 0 and N % 256 == 0):
        return False
    if schedule(form, M, N, K, torch.bfloat16) != 4:
        return False
    a_kc, b_kc = _KC[form]
    t = _TAIL.get((form, M, N, K, "bf16"), 0)
    if t and alpha_t is None:  # the tail-balanced launch, as ``mm`` takes it (its split part sums per tile)
        return bool(native().gemm8_tail(a, a_kc, b, b_kc, out, abs(t), t < 0, 4, sq))
    return bool(native().gemm8_sq(a, a_kc, b, b_kc, out, sq, alpha_t, 1.0))
