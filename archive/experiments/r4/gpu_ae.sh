#!/bin/bash
# round 4 pass AE: counted end-of-tile wait as the default -- attention + model tests at the default,
# kernel A/B at B16 and at one 8k sequence (17 = the old default)
OUT=gpurun_out/r4ae; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py -k "attention or attn or train_step or determin" -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
for i in 1 2; do
  for P in 17 273; do
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $OUT/b16_${P}_$i.txt 2>&1 || { echo "b16 $P rc=$?"; exit 1; }
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 120 python -u bench/attn_bench.py 1 32 8 8192 128 lite > $OUT/s8k_${P}_$i.txt 2>&1 || { echo "s8k $P rc=$?"; exit 1; }
    echo "prio $P run $i: B16 $(python -c "import json;j=json.loads(open('$OUT/b16_${P}_$i.txt').read().strip().splitlines()[-1]);print(j['bwd_ms'])") S8k $(python -c "import json;j=json.loads(open('$OUT/s8k_${P}_$i.txt').read().strip().splitlines()[-1]);print(j['bwd_ms'])")"
  done
done
