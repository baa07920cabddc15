#!/bin/bash
# Round-5 GPU pass M: SwiGLU backward in the down projection's dX GEMM epilogue (G8_EPI_SWIGLU_BWD):
# parity (epilogue vs fp32 and vs the two-step kernels, model bitwise), then config-2 and config-4
# proxy A/B against MXLLM_FUSED_SWIGLU_BWD=0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5m
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_fused_epi_gpu.py "tests/test_kernels_gpu.py::test_swiglu" "tests/test_kernels_gpu.py::test_swiglu_lora_tail" "tests/test_model_gpu.py::test_swiglu_recompute_bitwise_gpu" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for F in 0 1; do
    MXLLM_FUSED_SWIGLU_BWD=$F timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_f${F}_$i.json > $O/c2_f${F}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "c2 fused_bwd=$F run $i: $(python -c "import json;j=json.load(open('$O/c2_f${F}_$i.json'));print(j['value'],j['ms_per_step'],j['final_loss'])")"
  done
done
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
for F in 0 1; do
  MXLLM_FUSED_SWIGLU_BWD=$F timeout -k 10 400 python -u bench.py $C4 --json-out $O/c4_f$F.json > $O/c4_f$F.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
  echo "c4 fused_bwd=$F: $(python -c "import json;j=json.load(open('$O/c4_f$F.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_reserved_gb'],j['final_loss'])")"
done
echo done
