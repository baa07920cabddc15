#!/bin/bash
# 70B LoRA step: workgroup target of the rank-r kernels' split reduction (MXLLM_LORA_WGS).
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in ${WGS_LIST:-256 512 1024}; do
    MXLLM_LORA_WGS=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r2s3_wgs${v}_$i.json 2>/dev/null
  done
done
