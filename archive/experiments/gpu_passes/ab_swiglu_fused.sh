#!/bin/bash
# 8B decode: SwiGLU fused into the down projection vs separate kernels (same box, alternating).
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 0; do
    MXLLM_SWIGLU_FUSED=$v timeout -k 10 200 python bench/serve_bench.py --model llama3.1-8b --batches 1,8,64 \
      --requests 4 --new-tokens 4 > gpurun_out/r2s3_swi${v}_$i.json 2>/dev/null
  done
done
