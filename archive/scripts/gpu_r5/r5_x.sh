#!/bin/bash
# Round-5 GPU pass X: headline A/B of the in-launch LoRA split-K reduction (MXLLM_LORA_FUSED_RED=1, measured
# slower in round 3 with older kernels) -- LoRA tests with it on first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5x
mkdir -p $O
export PYTHONUNBUFFERED=1
MXLLM_LORA_FUSED_RED=1 timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "lora" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for F in 0 1; do
    MXLLM_LORA_FUSED_RED=$F timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/head_f${F}_$i.json > $O/head_f${F}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    echo "fused_red=$F run $i: $(python -c "import json;j=json.load(open('$O/head_f${F}_$i.json'));print(j['value'],j['ms_per_step'],j['final_loss'])")"
  done
done
echo done
