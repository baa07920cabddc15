#!/bin/bash
# round 4 pass T: swiglu_bwd_m (one pass over gu for dgu + the recomputed m) -- kernel / model tests,
# then the same-box config-4 A/B (m saved vs recomputed) at 40 and the planner's 16
OUT=gpurun_out/r4t; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "swiglu or recompute or train_step" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
run() {  # name recompute ck
  C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers $3 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
  MXLLM_RECOMPUTE_SWIGLU=$2 timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/$1.json > $OUT/$1.log 2>&1 || { echo "$1 rc=$?"; tail -3 $OUT/$1.log; return 1; }
  echo "$1: $(python -c "import json;j=json.load(open('$OUT/$1.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])")"
}
run ck40_saved 0 40 && run ck40_rec auto 40 && run ck16_rec auto 16 && run ck40_saved_b 0 40 && run ck40_rec_b auto 40 && run ck16_rec_b auto 16
