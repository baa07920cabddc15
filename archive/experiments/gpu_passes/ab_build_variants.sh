#!/bin/bash
# Same-box A/B of two builds of the native library: $1 = alternate .so (MXLLM_NATIVE_LIB), $2 = label;
# 8B decode at batches 1/8/64, alternating, two repeats.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench/serve_bench.py --model llama3.1-8b --batches 1,8,64 --requests 4 --new-tokens 4 \
    > gpurun_out/${2}_new_$i.json 2>/dev/null
  MXLLM_NATIVE_LIB=$1 timeout -k 10 200 python bench/serve_bench.py --model llama3.1-8b --batches 1,8,64 \
    --requests 4 --new-tokens 4 > gpurun_out/${2}_old_$i.json 2>/dev/null
done
