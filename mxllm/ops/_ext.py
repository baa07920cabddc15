"""Loader for the in-tree native library ``mxllm/_C.so`` (HIP kernels for gfx950).

Policy (MI355X-first, no silent fallbacks):
  * GPU tensors ALWAYS go through the HIP kernels.  If the library cannot be
    loaded on a machine with a GPU, ``native()`` raises — it never quietly
    substitutes an eager PyTorch path.
  * CPU tensors use the pure-PyTorch reference implementations in
    ``mxllm.ops.reference`` (used by the CPU test-suite / gloo plumbing runs and
    as numerics oracles for the kernel tests).
  * ``MXLLM_REFERENCE_OPS=1`` forces the reference path everywhere (debug only).
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_LOADED = False
_ERR: str | None = None
LIB = os.environ.get("MXLLM_NATIVE_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "_C.so")  # MXLLM_NATIVE_LIB: A/B builds only


def _load() -> bool:
    global _LOADED, _ERR
    if _LOADED:
        return True
    with _LOCK:
        if _LOADED:
            return True
        try:
            if not os.path.exists(LIB) and os.environ.get("MXLLM_NO_AUTOBUILD") != "1":
                from mxllm import _build

                _build.build()
            torch.ops.load_library(LIB)
            _LOADED = True
        except Exception as e:  # noqa: BLE001
            _ERR = f"{type(e).__name__}: {e}"
            _LOADED = False
    return _LOADED


def available() -> bool:
    return _load()


def native():
    """Return ``torch.ops.mxllm``; raise if the HIP library is unavailable."""
    if not _load():
        raise RuntimeError(
            "mxllm native library failed to load (" + str(_ERR) + "). Build it with "
            "`python -m mxllm._build` (hipcc --offload-arch=gfx950)."
        )
    return torch.ops.mxllm


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` must take the HIP path (any GPU tensor)."""
    if os.environ.get("MXLLM_REFERENCE_OPS") == "1":
        return False
    return t.is_cuda


def rows_view(t: torch.Tensor) -> torch.Tensor:
    """``t`` if it is a 2-D row-strided view the kernels accept (unit inner
    stride, row stride a multiple of 8: e.g. the left part of a padded
    buffer), otherwise a contiguous copy."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] and t.stride(0) % 8 == 0:
        return t
    return t.contiguous()
