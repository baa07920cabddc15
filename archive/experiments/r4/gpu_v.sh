#!/bin/bash
# round 4 pass V: LoRA rank-r kernels' workgroup target (MXLLM_LORA_WGS) swept at the 70B shapes:
# the lora_xtg grids of 288 / 576 tiles leave a short last wave at the 256-workgroup target
OUT=gpurun_out/r4v; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/lora_probe.py --wgs 0,256,512,1024,2304 --rounds 5 --json-out $OUT/lora_probe.json > $OUT/lora_probe.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/lora_probe.txt; exit 1; }
cat $OUT/lora_probe.txt
