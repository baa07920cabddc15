"""Per-step kernel time breakdown from a rocprofv3 kernel trace: the window
between the last two launches of a once-per-step kernel (the embedding lookup) -> one step.
usage: python scripts/step_breakdown.py <run_kernel_trace.csv> [top] [marker]
marker: kernel-name substring launched once per step (default: ``embedding_fwd``, else the grad-norm
or AdamW kernel)."""
import collections
import csv
import sys


def _rows(path: str) -> list[dict]:
    """Kernel rows from a rocprofv3 CSV kernel trace, or from its SQLite output (``*.db``, the
    default ``rocpd`` format): Kernel_Name / Start_Timestamp / End_Timestamp."""
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3

    con = sqlite3.connect(path)
    q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    return [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b} for n, a, b in con.execute(q)]


def main():
    rows = _rows(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a kernel launched once per step: the embedding lookup that opens every forward (the clip norm can
    # run as several partial passes per step, AdamW as several chunk launches)
    names = [r["Kernel_Name"] for r in rows]
    key = next((k for k in ("embedding_fwd", "sqnorm_partial", "adamw_kernel") if any(k in n for n in names)),
               "adamw_kernel")
    if len(sys.argv) > 3:
        key = sys.argv[3]
    marks = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    win = rows[a + 1:b + 1]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        n = r["Kernel_Name"]
        key = n.split("(")[0][:90]
        agg[key][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[key][1] += 1
    busy = sum(v[0] for v in agg.values())
    print(f"step window {1e-6 * (t1 - t0):.2f} ms, kernel busy {1e-6 * busy:.2f} ms, {len(win)} launches")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{1e-6 * t:9.3f} ms {c:6d}  {100 * t / busy:5.1f}%  {k}")


if __name__ == "__main__":
    main()
