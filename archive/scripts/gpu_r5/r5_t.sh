#!/bin/bash
# Round-5 GPU pass T: the clip norm from the dW GEMMs' per-tile sums of squares (gemm8_sq): kernel and
# trainer parity, the train / gemm8 suites, config-2 A/B against MXLLM_FUSED_GRAD_NORM=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5t
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gemm8_gpu.py tests/test_train_gpu.py tests/test_fused_epi_gpu.py tests/test_determinism_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for F in 0 1; do
    MXLLM_FUSED_GRAD_NORM=$F timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_f${F}_$i.json > $O/c2_f${F}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "c2 fused_norm=$F run $i: $(python -c "import json;j=json.load(open('$O/c2_f${F}_$i.json'));print(j['value'],j['ms_per_step'],j['final_loss'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py $C2 > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python $R/scripts/step_breakdown.py $O/prof/run_kernel_trace.csv 40 > $O/c2_breakdown.txt
rm -f $O/prof/run_kernel_trace.csv
head -12 $O/c2_breakdown.txt; grep -E "sqnorm|gemm8_kernel<false, false" $O/c2_breakdown.txt
echo done
