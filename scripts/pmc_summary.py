"""Summarise rocprofv3 --pmc counter CSVs per kernel (median over dispatches).
usage: python scripts/pmc_summary.py <dir-with-*_counter_collection.csv> [name-filter ...]"""
import collections
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    filt = sys.argv[2:]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if filt and not any(x in name for x in filt):
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            vals[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    for name, cs in vals.items():
        print(name[:100])
        for c, lst in sorted(cs.items()):
            per = collections.defaultdict(float)
            for did, v in lst:
                per[did] += v  # sum over dimensions (XCD/SE) of one dispatch
            print(f"   {c:28s} {statistics.median(per.values()):.4g}  (n={len(per)})")


if __name__ == "__main__":
    main()
