#!/bin/bash
# Round-5 GPU pass M2: config-2 kernel breakdown with / without the SwiGLU-backward epilogue
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5m2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off"
for F in 0 1; do
  MXLLM_FUSED_SWIGLU_BWD=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f$F -o run -- python3 $R/bench.py $C2 > $O/prof_f$F.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  python $R/scripts/step_breakdown.py $O/prof_f$F/run_kernel_trace.csv 40 > $O/c2_f${F}_breakdown.txt
  rm -f $O/prof_f$F/run_kernel_trace.csv
  head -14 $O/c2_f${F}_breakdown.txt
done
echo done
