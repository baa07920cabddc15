#!/bin/bash
# r6 pass H: same-box A/B of the headline with the lora_xtg wave-tile form on / off (alternating)
set -o pipefail
OUT=gpurun_out/r6h; mkdir -p $OUT
for run in 1 0 1 0; do
  tag=wt${run}_$((++i))
  MXLLM_LORA_XTG_WT=$run timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --config2 off --no-calibrate --json-out $OUT/head_$tag.json > $OUT/head_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 $OUT/head_$tag.log; exit 1; }
  echo "$tag: $(python -c "import json;j=json.load(open('$OUT/head_$tag.json'));print(j['value'],j['ms_per_step'],j['gpu_after_timed_steps'])")"
done
