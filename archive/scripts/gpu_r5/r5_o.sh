#!/bin/bash
# Round-5 GPU pass O: SwiGLU-backward epilogue with its gu loads batched per half-tile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5o
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_fused_epi_gpu.py "tests/test_model_gpu.py::test_swiglu_recompute_bitwise_gpu" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
cd /tmp && export TMPDIR=/tmp
C2="--model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off"
for F in 1 0; do
  MXLLM_FUSED_SWIGLU_BWD=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f$F -o run -- python3 $R/bench.py $C2 > $O/prof_f$F.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  python $R/scripts/step_breakdown.py $O/prof_f$F/run_kernel_trace.csv 40 > $O/c2_f${F}_breakdown.txt
  rm -f $O/prof_f$F/run_kernel_trace.csv
  head -1 $O/c2_f${F}_breakdown.txt; grep -E "gemm8_kernel<true, false, false, false, 0, 4, [03]>|swiglu_bwd" $O/c2_f${F}_breakdown.txt
done
cd $R
for i in 1 2; do
  for F in 0 1; do
    MXLLM_FUSED_SWIGLU_BWD=$F timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_f${F}_$i.json > $O/c2_f${F}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "c2 fused_bwd=$F run $i: $(python -c "import json;j=json.load(open('$O/c2_f${F}_$i.json'));print(j['value'],j['ms_per_step'],j['final_loss'])")"
  done
done
echo done
