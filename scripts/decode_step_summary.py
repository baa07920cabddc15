"""Per-kernel breakdown of the median graphed decode step in a rocprofv3 kernel trace
(embedding -> sample); usage: decode_step_summary.py <run_kernel_trace.csv>."""
import collections
import csv
import sys


def step_summary(path: str) -> str:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    emb = [i for i, r in enumerate(rows) if "embedding_fwd" in r["Kernel_Name"]]
    stats = []
    for a, b in zip(emb, emb[1:]):
        seg = rows[a:b]
        names = [r["Kernel_Name"] for r in seg]
        if not any("decode_attn" in n for n in names) or any("attn_fwd" in n for n in names):
            continue  # not a decode step (prefill)
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
        stats.append((t1 - t0, busy, len(seg), a, b))
    stats.sort()
    w, busy, n, a, b = stats[len(stats) // 2]
    out = [f"median graphed decode step (embedding -> sample): wall {w / 1e3:.1f} us, "
           f"kernel busy {busy / 1e3:.1f} us, {n} kernels"]
    tot = collections.defaultdict(lambda: [0, 0])
    for r in rows[a:b]:
        k = r["Kernel_Name"].split("(")[0][:70]
        tot[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[k][1] += 1
    for k, (d, c) in sorted(tot.items(), key=lambda x: -x[1][0]):
        out.append(f"{d / 1e3:9.1f} us {c:4d}  {k}")
    return "\n".join(out)


if __name__ == "__main__":
    print(step_summary(sys.argv[1]))
