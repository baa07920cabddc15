"""Per-shape hipBLASLt/rocBLAS solution selection via PyTorch TunableOp.

The GEMMs stay plain library calls; TunableOp only picks, per (op, shape),
the fastest solution among hipBLASLt's and rocBLAS's own kernels.  The
selection table ``mxllm/tuning/tunableop_gfx950.csv`` was measured on MI355X
(bench/tune_gemms.py) and is used read-only: tuning is OFF at run time, and
shapes not in the table fall back to the library default.  Measured effect on
the Llama-3.1-70B QKV projection (4096x8192 -> 10240): 952 -> 1433 TFLOP/s
forward, 1078 -> 1366 TFLOP/s for dX.
"""
from __future__ import annotations

import logging
import os

import torch

log = logging.getLogger("mxllm.gemm")
TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "tunableop_gfx950.csv")
_ON = False


def enable(path: str | None = None) -> bool:
    """Use the tuned GEMM table (read-only; ``MXLLM_GEMM_TABLE`` overrides the
    path).  No-op without a GPU / table or when MXLLM_GEMM_TUNING=0."""
    global _ON
    path = path or os.environ.get("MXLLM_GEMM_TABLE") or TABLE
    if _ON:
        return True
    if os.environ.get("MXLLM_GEMM_TUNING", "1") == "0" or not torch.cuda.is_available() or not os.path.exists(path):
        return False
    try:
        import shutil
        import tempfile

        # work on a private copy: TunableOp may rewrite its file at exit
        tmp = os.path.join(tempfile.gettempdir(), f"mxllm_tunableop_{os.getpid()}.csv")
        shutil.copyfile(path, tmp)
        tun = torch.cuda.tunable
        tun.enable(True)
        tun.tuning_enable(False)
        if hasattr(tun, "record_untuned_enable"):
            tun.record_untuned_enable(False)
        tun.set_filename(tmp, insert_device_ordinal=False)
        ok = tun.read_file(tmp)
        _ON = bool(ok) or ok is None
    except Exception as e:  # noqa: BLE001
        log.warning("TunableOp table not used: %s", e)
        return False
    return True
