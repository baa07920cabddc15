"""Profiling helpers: roctx ranges emitted by the native
library (``csrc/runtime/roctx.cpp`` -> rocprofiler-sdk roctx, visible in
``rocprofv3 --marker-trace``) and a step timer using HIP events.

Ranges are on by default on GPU and cost one C call each; ``MXLLM_ROCTX=0``
turns them off.
"""
from __future__ import annotations

import contextlib
import os

import torch

_ON: bool | None = None


def _enabled() -> bool:
    global _ON
    if _ON is None:
        _ON = False
        if os.environ.get("MXLLM_ROCTX", "1") != "0" and torch.cuda.is_available():
            try:
                from ..ops._ext import native

                native()
                _ON = bool(torch.ops.mxllm.roctx_available())
            except Exception:  # noqa: BLE001
                _ON = False
    return _ON


def set_enabled(flag: bool) -> None:
    """Turn ranges off, or back on (re-probing the native library)."""
    global _ON
    _ON = False if not flag else None


@contextlib.contextmanager
def range_(name: str):
    """``with range_("backward"): ...`` — a named roctx range (no-op on CPU)."""
    if not _enabled():
        yield
        return
    torch.ops.mxllm.roctx_push(name)
    try:
        yield
    finally:
        torch.ops.mxllm.roctx_pop()


def mark(name: str) -> None:
    if _enabled():
        torch.ops.mxllm.roctx_mark(name)


class EventTimer:
    """Device-side elapsed time between two points on the current stream."""

    def __init__(self):
        self.enabled = torch.cuda.is_available()
        if self.enabled:
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)

    def start(self):
        if self.enabled:
            self.a.record()

    def stop(self) -> float:
        if not self.enabled:
            return 0.0
        self.b.record()
        self.b.synchronize()
        return self.a.elapsed_time(self.b)
