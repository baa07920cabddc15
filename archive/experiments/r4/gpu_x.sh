#!/bin/bash
# round 4 pass X: fp8 decode GEMM channel groups per wave (MXLLM_W8_NC) at the 70B / 8B shapes
OUT=gpurun_out/r4x; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/w8_probe.py --json-out $OUT/w8_probe.json > $OUT/w8_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/w8_probe.txt; exit 1; }
cat $OUT/w8_probe.txt
