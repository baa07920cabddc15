#!/bin/bash
# round 4 pass AD: attention backward, counted end-of-tile wait (MXLLM_ATTN_BWD8_PRIO bit 256: the dS^T
# stores stay in flight across the barrier) -- attention tests with it, kernel A/B, headline A/B
OUT=gpurun_out/r4ad; mkdir -p $OUT
export PYTHONUNBUFFERED=1
MXLLM_ATTN_BWD8_PRIO=273 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or attn or train_step" -x -v --timeout 120 --timeout-method thread > $OUT/tests_273.txt 2>&1
rc=$?; tail -2 $OUT/tests_273.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
for i in 1 2 3; do
  for P in 17 273; do
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/attn_${P}_$i.txt 2>&1 || { echo "attn $P rc=$?"; exit 1; }
    echo "prio $P run $i: $(grep shape $OUT/attn_${P}_$i.txt)"
  done
done
for i in 1 2; do
  for P in 17 273; do
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 400 python bench.py --config2 off --no-calibrate > $OUT/bench_${P}_$i.json 2> $OUT/bench_${P}_$i.err || { echo "bench $P rc=$?"; exit 1; }
    echo "headline prio $P run $i: $(python -c "import json;print(json.load(open('$OUT/bench_${P}_$i.json'))['ms_per_step'])")"
  done
done
