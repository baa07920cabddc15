"""Per-call durations of one kernel inside one training step, grouped by launch shape.

usage: python scripts/kernel_calls.py <run_kernel_trace.csv> <kernel-substring> [marker]

The step window is the one ``scripts/step_breakdown.py`` uses (between the last two launches of a
once-per-step kernel, ``marker``, default ``embedding_fwd``).  Calls of the kernel are grouped by
(grid, workgroup) size -- e.g. the LoRA ``lora_xtg`` launches of the q/k/v, o, gate-up and down
projections -- and each group prints count, total, mean and min microseconds, so a slow projection
shape stands out.
"""
import collections
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    marker = sys.argv[3] if len(sys.argv) > 3 else "embedding_fwd"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit(f"fewer than two {marker!r} launches in the trace")
    win = rows[marks[-2] + 1:marks[-1] + 1]
    groups = collections.defaultdict(list)
    for r in win:
        if name not in r["Kernel_Name"]:
            continue
        key = (r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""),
               r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?")))
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in groups.values())
    print(f"{name}: {sum(len(v) for v in groups.values())} calls, {tot / 1e3:.3f} ms in the step")
    for key, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"  grid {key[0]}x{key[1] or 1} wg {key[2]}: {len(v):4d} calls  total {sum(v) / 1e3:8.3f} ms  "
              f"mean {sum(v) / len(v):8.1f} us  min {min(v):8.1f} us")


if __name__ == "__main__":
    main()
