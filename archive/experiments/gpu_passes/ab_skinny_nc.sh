#!/bin/bash
# 8B decode: channel groups per workgroup of the plain decode GEMM (o / down / LM head), same box.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 2 4; do
    MXLLM_SKINNY_NC=$v timeout -k 10 200 python bench/serve_bench.py --model llama3.1-8b --batches 1,4,8 \
      --requests 4 --new-tokens 4 > gpurun_out/r2s3_nc${v}_$i.json 2>/dev/null
  done
done
