#!/bin/bash
# round 4 pass Z: decode GEMMs at 1..64 token rows (70B / 8B shapes): hipBLASLt vs the skinny HIP
# kernel at 1 / 2 / 4 channel groups (MXLLM_SKINNY_NC) -- is there a medium-batch decode gap?
OUT=gpurun_out/r4z; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for NC in 1 2 4; do
  MXLLM_SKINNY_NC=$NC timeout -k 10 300 python -u bench/skinny_gemm_probe.py 70b,8b > $OUT/probe_nc$NC.jsonl 2>&1 || { echo "probe nc$NC rc=$?"; tail -3 $OUT/probe_nc$NC.jsonl; exit 1; }
done
echo done
