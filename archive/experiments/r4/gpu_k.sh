#!/bin/bash
# round 4 pass K: lora_xwt split reduction over 16-row workgroups (4x the grid) vs 64-row
OUT=gpurun_out/r4k; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -v --timeout 120 --timeout-method thread > $OUT/tests_kernel.txt 2>&1
rc=$?; tail -2 $OUT/tests_kernel.txt; [ $rc -eq 0 ] || { echo "kernel tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench/lora_probe.py --rounds 5 --json-out $OUT/lora_probe.json > $OUT/lora_probe.txt 2>&1 || { echo "lora probe rc=$?"; exit 1; }
grep xwt $OUT/lora_probe.txt | cut -c1-200
for i in 1 2; do
  MXLLM_LORA_XWT_RED_ROWS=64 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "red64 $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'])")  red16 $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'])")"
done
