"""Env/config-driven fault injection for failure-detection drills.

MXLLM_FAULT_RANK / MXLLM_FAULT_STEP / MXLLM_FAULT_KIND (exit | raise | hang | nan):
the selected rank misbehaves at the selected step.  Used by the fault tests to
prove jobs fail fast and cleanly (no hang) and that --max-restarts + checkpoint
resume recovers.  A restarted worker (TORCHELASTIC_RESTART_COUNT > 0) does not
re-inject, so the drill converges.
"""
from __future__ import annotations

import logging
import os
import time

log = logging.getLogger("mxllm.faults")


class InjectedFault(RuntimeError):
    pass


def maybe_inject(cfg, rank: int, step: int) -> None:
    fr, fs, kind = getattr(cfg, "fault_rank", -1), getattr(cfg, "fault_step", -1), getattr(cfg, "fault_kind", "")
    if not kind or fr != rank or fs != step:
        return
    if int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0 and os.environ.get("MXLLM_FAULT_ON_RESTART") != "1":
        return
    log.error("[rank %d] injecting fault %r at step %d", rank, kind, step)
    if kind == "exit":
        os._exit(13)
    if kind == "raise":
        raise InjectedFault(f"injected fault at rank {rank} step {step}")
    if kind == "hang":
        deadline = time.time() + float(os.environ.get("MXLLM_FAULT_HANG_S", "3600"))
        while time.time() < deadline:
            time.sleep(0.5)
    if kind == "nan":
        raise FloatingPointError(f"injected non-finite loss at rank {rank} step {step}")
