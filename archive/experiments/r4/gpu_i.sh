#!/bin/bash
# round 4 pass I: row-tiled lora_xwt (adapter rows only, 64 token rows per workgroup): numerics,
# speed vs the LDS-DMA kernel per 70B projection, headline A/B
OUT=gpurun_out/r4i; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -v --timeout 120 --timeout-method thread > $OUT/tests_kernel.txt 2>&1
rc=$?; tail -3 $OUT/tests_kernel.txt; [ $rc -eq 0 ] || { echo "kernel tests rc=$rc"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -k "lora or train_step" -x -v --timeout 120 --timeout-method thread > $OUT/tests_model.txt 2>&1
rc=$?; tail -3 $OUT/tests_model.txt; [ $rc -eq 0 ] || { echo "model tests rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench/lora_probe.py --rounds 5 --json-out $OUT/lora_probe.json > $OUT/lora_probe.txt 2>&1 || { echo "lora probe rc=$?"; exit 1; }
cut -c1-300 $OUT/lora_probe.txt
for i in 1 2; do
  MXLLM_LORA_XWT=lds timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "lds $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'])")  tile $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'])")"
done
