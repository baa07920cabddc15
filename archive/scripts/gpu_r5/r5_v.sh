#!/bin/bash
# Round-5 GPU pass V: config-2 kernel breakdown at the final tree (embedding_fwd as the step marker)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py $C2 > $O/prof_c2.log 2>&1 || { echo "prof c2 rc=$?"; exit 1; }
python $R/scripts/step_breakdown.py $O/prof_c2/run_kernel_trace.csv 40 > $O/step_breakdown_c2_8b_full.txt
rm -f $O/prof_c2/run_kernel_trace.csv
head -24 $O/step_breakdown_c2_8b_full.txt
echo done
