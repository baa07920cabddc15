#!/bin/bash
# Round-5 GPU pass Y: config 2 vs the overlapped AdamW's grid cap (MXLLM_ADAMW_GRID: fewer AdamW workgroups
# beside the forward GEMMs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5y
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for G in 2048 1024 512; do
    MXLLM_ADAMW_GRID=$G timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_g${G}_$i.json > $O/c2_g${G}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "adamw_grid=$G run $i: $(python -c "import json;j=json.load(open('$O/c2_g${G}_$i.json'));print(j['value'],j['ms_per_step'])")"
  done
done
echo done
