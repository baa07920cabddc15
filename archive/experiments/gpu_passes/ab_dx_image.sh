#!/bin/bash
# A/B of the transposed [W; A] dX image (MXLLM_DX_IMAGE) on the 70B LoRA headline, same box.
set -e
O=gpurun_out/abdx2; mkdir -p $O
for v in none o qkv,o o; do
  MXLLM_DX_IMAGE=${v/none/} timeout -k 10 400 python bench.py --steps 6 --warmup 2 --json-out $O/$v.json > $O/$v.log 2>&1
  python -c "import json;d=json.load(open('$O/$v.json'));print('$v',d['value'],d['ms_per_step'],d['peak_hbm_gb'])" >> $O/summary.txt
done
