"""Re-tune the hipBLASLt/rocBLAS solution choice for EVERY GEMM a bench workload issues.

Runs ``bench.run`` for a few steps with PyTorch TunableOp tuning ON (each new (op, shape,
layout, dtype) is timed over the libraries' own solutions, the fastest is recorded), then
merges the result with the committed table (``mxllm/tuning/tunableop_gfx950.csv``): new
shapes are added, shapes already there keep the faster of the two recorded times.  The
GEMMs stay plain library calls; the table only selects among hipBLASLt's / rocBLAS's own
kernels.  usage (GPU box):
  python bench/tune_headline.py --out gpurun_out/tune/merged.csv [bench args...]
"""
from __future__ import annotations

import argparse
import csv
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def merge(old_path: str, new_path: str, out_path: str) -> dict:
    def rows(p):
        out = {}
        hdr = []
        if not os.path.exists(p):
            return hdr, out
        for r in csv.reader(open(p)):
            if not r:
                continue
            if r[0] == "Validator":
                hdr.append(r)
            elif len(r) >= 4:
                out[(r[0], r[1])] = r
        return hdr, out

    h_old, old = rows(old_path)
    h_new, new = rows(new_path)
    merged = dict(old)
    stats = {"old": len(old), "new": len(new), "added": 0, "replaced": 0}
    for k, r in new.items():
        if k not in merged:
            merged[k] = r
            stats["added"] += 1
        elif float(r[3]) < float(merged[k][3]):
            merged[k] = r
            stats["replaced"] += 1
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        for r in (h_old or h_new):
            w.writerow(r)
        for r in merged.values():
            w.writerow(r)
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-ms", type=int, default=60, help="tuning time budget per GEMM shape")
    ap.add_argument("--base", default=os.path.join(ROOT, "mxllm", "tuning", "tunableop_gfx950.csv"),
                    help="table the new selections are merged into")
    a, rest = ap.parse_known_args()
    import bench
    from mxllm.parallel import runtime

    raw = a.out + ".raw.csv"
    import threading
    import time

    t0 = time.time()

    def heartbeat():  # tuning one large shape takes minutes: show progress (and stay alive)
        while True:
            time.sleep(20)
            try:
                n = len(torch.cuda.tunable.get_results())
            except Exception:  # noqa: BLE001
                n = -1
            print(f"[tune] {time.time() - t0:.0f} s, {n} GEMM shapes tuned so far", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_filename(raw, insert_device_ordinal=False)
    args = bench.parse(rest + ["--no-gemm-table", "--config2", "off", "--config3", "off", "--config4", "off"])
    env = runtime.init()
    out = bench.run(args, env)
    if hasattr(tun, "write_file"):
        tun.write_file(raw)
    else:  # torch >= 2.10: no write_file; write validators + results in the table's CSV format
        with open(raw, "w", newline="") as f:
            w = csv.writer(f)
            for v in tun.get_validators():
                w.writerow(["Validator", *v])
            for r in tun.get_results():
                w.writerow(list(r))
    stats = merge(a.base, raw, a.out)
    print({"tuned_run_ms_per_step": out["ms_per_step"], **stats}, flush=True)
    runtime.cleanup()


if __name__ == "__main__":
    main()
