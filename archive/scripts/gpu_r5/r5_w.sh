#!/bin/bash
# Round-5 GPU pass W: the final trainer / tail-launch changes (clip-norm partials from the tail-balanced
# launch too, one fixed-order sum of the parts): gemm8 / train / determinism / multi-rank suites, the
# config-2 A/B against MXLLM_FUSED_GRAD_NORM=0, a config-2 kernel breakdown, the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5w
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_train_gpu.py tests/test_determinism_gpu.py tests/test_multirank_gpu.py tests/test_gemm8_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for F in 0 1; do
    MXLLM_FUSED_GRAD_NORM=$F timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_f${F}_$i.json > $O/c2_f${F}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "c2 fused_norm=$F run $i: $(python -c "import json;j=json.load(open('$O/c2_f${F}_$i.json'));print(j['value'],j['ms_per_step'],j['final_loss'])")"
  done
done
ROOT=$R
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $ROOT/bench.py $C2 > $O/prof_c2.log 2>&1 || { echo "prof c2 rc=$?"; exit 1; }
python $ROOT/scripts/step_breakdown.py $O/prof_c2/run_kernel_trace.csv 40 > $O/step_breakdown_c2_8b_full.txt
rm -f $O/prof_c2/run_kernel_trace.csv
head -3 $O/step_breakdown_c2_8b_full.txt; grep -E "sqnorm|g8_sum2" $O/step_breakdown_c2_8b_full.txt
cd $ROOT
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$O/bench.json'));print(j['value'],j['ms_per_step'],j['config2_8b_full']['value'],j['config2_8b_full']['ms_per_step'],j['calibration'])"
echo done
