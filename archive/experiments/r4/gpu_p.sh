#!/bin/bash
# round 4 pass P: SwiGLU-LoRA kernel with 2 / 4 row blocks per workgroup sharing the V fragments
OUT=gpurun_out/r4p; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "swiglu" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench/swiglu_lora_probe.py --cs 0,1,2 --rbw 1,2,4 --rounds 5 --json-out $OUT/probe.json > $OUT/probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
cut -c1-1200 $OUT/probe.txt
for i in 1 2; do
  MXLLM_SWIGLU_LORA_RBW=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_r1_$i.json 2> $OUT/bench_r1_$i.err || { echo "bench rc=$?"; exit 1; }
  MXLLM_SWIGLU_LORA_RBW=2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_r2_$i.json 2> $OUT/bench_r2_$i.err || { echo "bench rc=$?"; exit 1; }
  MXLLM_SWIGLU_LORA_RBW=4 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_r4_$i.json 2> $OUT/bench_r4_$i.err || { echo "bench rc=$?"; exit 1; }
  echo "rbw1 $i: $(python -c "import json;j=json.load(open('$OUT/bench_r1_$i.json'));print(j['ms_per_step'])")  rbw2: $(python -c "import json;j=json.load(open('$OUT/bench_r2_$i.json'));print(j['ms_per_step'])")  rbw4: $(python -c "import json;j=json.load(open('$OUT/bench_r4_$i.json'));print(j['ms_per_step'])")"
done
