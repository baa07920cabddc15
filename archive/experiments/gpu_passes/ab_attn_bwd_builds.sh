#!/bin/bash
# A/B of backward-attention build variants (build_ab/<V>/_C.so): numerics then the microbenchmark.
set -e
for V in "$@"; do
  MXLLM_NATIVE_LIB=build_ab/$V/_C.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2r_tests_$V.log 2>&1
  MXLLM_NATIVE_LIB=build_ab/$V/_C.so timeout -k 10 120 python bench/attn_bench.py > gpurun_out/r2r_attn_$V.json 2>/dev/null
done
