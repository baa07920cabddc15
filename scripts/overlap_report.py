"""Optimizer/compute overlap in a rocprofv3 kernel trace (round 3).

Steps are delimited by the one grad-norm kernel per step (``sqnorm_partial``).
For each step window this reports the wall time, the summed fused-AdamW kernel
time, how much of it ran concurrently with any other kernel (interval
intersection across queues) and how much was EXPOSED (AdamW the only kernel on
the device).
usage: python scripts/overlap_report.py <run_kernel_trace.csv> [more.csv ...]
"""
import csv
import sys


def _merge(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _inter(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def report(path):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    marks = [k[0] for k in ks if "sqnorm_partial" in k[2]]
    print(f"== {path}: {len(ks)} kernels, {len(marks)} steps")
    for s0, s1 in zip(marks, marks[1:]):
        win = [k for k in ks if s0 <= k[0] < s1]
        adam = [(a, b) for a, b, n in win if "adamw_kernel" in n]
        other = _merge([(a, b) for a, b, n in win if "adamw_kernel" not in n])
        tot = sum(b - a for a, b in adam)
        ov = _inter(_merge(adam), other)
        print(f"step {1e-6 * (s1 - s0):8.2f} ms | adamw {len(adam):3d} launches {1e-6 * tot:7.2f} ms busy, "
              f"{1e-6 * ov:7.2f} ms concurrent with other kernels, {1e-6 * (_span(adam) - ov):7.2f} ms exposed")


def _span(iv):
    return sum(b - a for a, b in _merge(iv))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        report(p)
