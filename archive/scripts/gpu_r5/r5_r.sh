#!/bin/bash
# Round-5 GPU pass R: copy2d_batched transposing copies through 64 x 64 LDS tiles (the LoRA B^T / A
# images refreshed after every optimizer step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5r
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_copy2d_gpu.py tests/test_model_gpu.py -k "copy2d or lora or adapter" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o run -- python3 $R/bench.py --steps 3 --warmup 1 --config2 off --no-calibrate > $O/prof_head.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python $R/scripts/step_breakdown.py $O/prof_head/run_kernel_trace.csv 40 > $O/step_breakdown_70b_lora.txt
rm -f $O/prof_head/run_kernel_trace.csv
head -1 $O/step_breakdown_70b_lora.txt; grep -E "copy2d" $O/step_breakdown_70b_lora.txt
echo done
