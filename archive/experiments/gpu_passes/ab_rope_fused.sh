#!/bin/bash
# Decode: RMSNorm in the GEMM prologue vs the separate RMSNorm kernel (same box, alternating).
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 0; do
    MXLLM_ROPE_FUSED=$v timeout -k 10 200 python bench/serve_bench.py --model llama3.1-8b --batches 1,2,4 \
      --requests 4 --new-tokens 4 > gpurun_out/r2s3_rf${v}_8b_$i.json 2>/dev/null
  done
done
for v in 1 0; do
  MXLLM_ROPE_FUSED=$v timeout -k 10 300 python bench/serve_bench.py --model llama3.1-70b --batches 1,2 \
    --requests 4 --new-tokens 4 > gpurun_out/r2s3_rf${v}_70b.json 2>/dev/null
done
