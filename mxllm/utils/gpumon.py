"""GPU monitoring through AMD SMI.

The reference's setup guide tells users to watch ``nvidia-smi`` by hand
(reference docs/setup_guide.md:71).  mxllm samples its own GPU from inside the
job: a daemon thread reads AMD SMI metrics for the device this rank is bound
to (matched by PCI bus id) — GFX / memory activity, clocks, socket power,
hotspot / HBM temperature, VRAM use, xGMI traffic counters — and hands each
sample to a callback (the fine-tune driver writes them to its JSONL metrics
as ``kind="gpu"`` records).  ``python -m mxllm.utils.gpumon`` prints the same
fields for every visible GPU (an ``amd-smi monitor`` equivalent).

Read-only: nothing here changes clocks, power caps or any GPU setting.
"""
from __future__ import annotations

import logging
import threading
import time

import torch

log = logging.getLogger("mxllm.gpumon")

# gpu_metrics_info keys worth logging (missing keys are skipped: firmware-dependent)
_KEYS = {
    "average_gfx_activity": "gfx_activity_pct",
    "average_umc_activity": "mem_activity_pct",
    "current_socket_power": "socket_power_w",
    "average_socket_power": "avg_socket_power_w",
    "temperature_hotspot": "temp_hotspot_c",
    "temperature_mem": "temp_hbm_c",
    "current_gfxclk": "gfx_clock_mhz",
    "current_uclk": "mem_clock_mhz",
    "xgmi_read_data_acc": "xgmi_read_kb",
    "xgmi_write_data_acc": "xgmi_write_kb",
}


def _bdf(index: int) -> str:
    p = torch.cuda.get_device_properties(index)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def _scalar(v, total: bool = False):
    """Per-XCD / per-link lists: summed for traffic counters, averaged otherwise."""
    if isinstance(v, (list, tuple)):
        vals = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF)]
        if not vals:
            return None
        return sum(vals) if total else round(sum(vals) / len(vals), 1)
    if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
        return v
    return None


class _Smi:
    _lock = threading.Lock()
    _refs = 0

    def __enter__(self):
        import amdsmi

        with _Smi._lock:
            if _Smi._refs == 0:
                amdsmi.amdsmi_init()
            _Smi._refs += 1
        return amdsmi

    def __exit__(self, *a):
        import amdsmi

        with _Smi._lock:
            _Smi._refs -= 1
            if _Smi._refs == 0:
                try:
                    amdsmi.amdsmi_shut_down()
                except Exception:  # noqa: BLE001
                    pass
        return False


def sample_handle(smi, h) -> dict:
    out = {}
    try:
        m = smi.amdsmi_get_gpu_metrics_info(h)
        for k, name in _KEYS.items():
            if k in m:
                v = _scalar(m[k], total=k.startswith("xgmi"))
                if v is not None:
                    out[name] = v
    except Exception as e:  # noqa: BLE001
        out["metrics_error"] = str(e)[:120]
    try:
        u = smi.amdsmi_get_gpu_vram_usage(h)
        out["vram_used_mb"] = u.get("vram_used")
        out["vram_total_mb"] = u.get("vram_total")
    except Exception:  # noqa: BLE001
        pass
    return out


def sample_device(index: int) -> dict:
    """One sample for ``cuda:index`` (empty dict when AMD SMI is unavailable)."""
    try:
        with _Smi() as smi:
            h = smi.amdsmi_get_processor_handle_from_bdf(_bdf(index))
            return sample_handle(smi, h)
    except Exception as e:  # noqa: BLE001
        log.debug("AMD SMI sample failed: %s", e)
        return {}


class GpuMonitor:
    """Background sampler: ``GpuMonitor(device, period_s, callback).start()``."""

    def __init__(self, device: torch.device, period_s: float, callback):
        self.device, self.period, self.cb = device, float(period_s), callback
        self._stop = threading.Event()
        self._t = None

    def start(self):
        if self.period <= 0 or self.device.type != "cuda":
            return self
        self._t = threading.Thread(target=self._run, name="mxllm-gpumon", daemon=True)
        self._t.start()
        return self

    def _run(self):
        try:
            with _Smi() as smi:
                h = smi.amdsmi_get_processor_handle_from_bdf(_bdf(self.device.index))
                while not self._stop.is_set():
                    s = sample_handle(smi, h)
                    s["hbm_allocated_gb"] = torch.cuda.memory_allocated(self.device) / 1e9
                    try:
                        self.cb(s)
                    except Exception as e:  # noqa: BLE001
                        log.debug("gpu monitor callback failed: %s", e)
                    self._stop.wait(self.period)
        except Exception as e:  # noqa: BLE001
            log.warning("GPU monitor disabled: %s", e)

    def stop(self):
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=5)
            self._t = None


def main():
    if not torch.cuda.is_available():
        print("no GPU visible")
        return
    rows = []
    for i in range(torch.cuda.device_count()):
        s = sample_device(i)
        rows.append((i, _bdf(i), s))
    for i, bdf, s in rows:
        fields = " ".join(f"{k}={v}" for k, v in s.items())
        print(f"cuda:{i} {bdf} {fields}")


if __name__ == "__main__":
    main()
