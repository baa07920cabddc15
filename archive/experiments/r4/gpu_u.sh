#!/bin/bash
# round 4 pass U: the normed qkv / gate-up inputs recomputed too (ops.normed_linear) -- tests, then
# the same-box config-4 proxy: 16 checkpointed with / without the norm recompute, 8, 0; 40 m saved
OUT=gpurun_out/r4u; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "swiglu or recompute or train_step" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
run() {  # name recompute-m recompute-norm ck
  C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers $4 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
  MXLLM_RECOMPUTE_SWIGLU=$2 MXLLM_RECOMPUTE_NORM=$3 timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/$1.json > $OUT/$1.log 2>&1 || { echo "$1 rc=$?"; tail -3 $OUT/$1.log; return 1; }
  echo "$1: $(python -c "import json;j=json.load(open('$OUT/$1.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])")"
}
run ck16_m auto 0 16 && run ck16_mx auto auto 16 && run ck8_mx auto auto 8 && run ck0_mx auto auto 0 && run ck40_saved 0 0 40
