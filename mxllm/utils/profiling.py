"""Profiling helpers: roctx ranges (visible in rocprofv3 --marker-trace) and a
step timer using HIP events.  ``torch.cuda.nvtx`` maps to roctx on ROCm builds."""
from __future__ import annotations

import contextlib

import torch


@contextlib.contextmanager
def range_(name: str):
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:  # noqa: BLE001
            yield
            return
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


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
