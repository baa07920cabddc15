#!/bin/bash
# Round-5 GPU pass P: config-2 kernel order around the generic strided copies (what issues them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 2 --warmup 1 --no-calibrate --config2 off"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py $C2 > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python - $O/prof/run_kernel_trace.csv > $O/copy_context.txt <<'P'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
for i, n in enumerate(names):
    if "direct_copy" in n or "bfloat16_copy" in n:
        d = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1000
        if d < 100 and "bfloat16_copy" in n:
            continue
        print(f"--- #{i} {d:.1f} us {n[:90]}")
        for j in range(max(0, i - 3), min(len(names), i + 4)):
            print("   ", j, names[j][:110])
P
head -80 $O/copy_context.txt
rm -f $O/prof/run_kernel_trace.csv
echo done
