"""Device<->host copies inside one optimizer step of a rocprofv3 trace: the window
between the last two fused-AdamW kernels.  A copy to the host inside that window
before the optimizer is a host synchronisation in the step.
usage: python scripts/step_copies.py <rocprofv3 output dir>"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    mc = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
    ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    ad = [int(r["Start_Timestamp"]) for r in ks if "adamw_kernel" in r["Kernel_Name"]]
    if len(ad) < 2:
        print("fewer than two optimizer steps in the trace")
        return
    t0, t1 = ad[-2], ad[-1]
    rows = list(csv.DictReader(open(mc[0]))) if mc else []
    inside = [r for r in rows if t0 < int(r["Start_Timestamp"]) < t1]
    d2h = [r for r in inside if "HOST" in r.get("Direction", "").split("_TO_")[-1]]
    print(f"step window {1e-6 * (t1 - t0):.2f} ms; copies inside: {len(inside)}; device->host: {len(d2h)}")
    for r in inside:
        print(f"  {r.get('Direction')} {r.get('Size', r.get('Bytes', '?'))} B at +{1e-6 * (int(r['Start_Timestamp']) - t0):.3f} ms")


if __name__ == "__main__":
    main()
