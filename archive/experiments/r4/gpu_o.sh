#!/bin/bash
# round 4 pass O: register-fragment SwiGLU-LoRA variant (no LDS image, no loop barrier) vs the LDS one
OUT=gpurun_out/r4o; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "swiglu" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench/swiglu_lora_probe.py --cs 0,4,8 --rounds 5 --json-out $OUT/probe.json > $OUT/probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
cut -c1-700 $OUT/probe.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_lds_$i.json 2> $OUT/bench_lds_$i.err || { echo "bench rc=$?"; exit 1; }
  MXLLM_SWIGLU_LORA_V=reg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_reg_$i.json 2> $OUT/bench_reg_$i.err || { echo "bench rc=$?"; exit 1; }
  echo "lds $i: $(python -c "import json;j=json.load(open('$OUT/bench_lds_$i.json'));print(j['ms_per_step'])")  reg $i: $(python -c "import json;j=json.load(open('$OUT/bench_reg_$i.json'));print(j['ms_per_step'])")"
done
