#!/bin/bash
# Round-5 GPU pass Z: the AdamW grid cap around its optimum (config 2), and its effect on the headline
# and on the config-4 proxy
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5z
mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for G in 2048 1536 1024 768; do
    MXLLM_ADAMW_GRID=$G timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/c2_g${G}_$i.json > $O/c2_g${G}_$i.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
    echo "c2 adamw_grid=$G run $i: $(python -c "import json;j=json.load(open('$O/c2_g${G}_$i.json'));print(j['value'],j['ms_per_step'])")"
  done
done
for G in 2048 1024; do
  MXLLM_ADAMW_GRID=$G timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-calibrate --config2 off --json-out $O/head_g$G.json > $O/head_g$G.log 2>&1 || { echo "head rc=$?"; exit 1; }
  echo "headline adamw_grid=$G: $(python -c "import json;j=json.load(open('$O/head_g$G.json'));print(j['value'],j['ms_per_step'])")"
done
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
for G in 2048 1024; do
  MXLLM_ADAMW_GRID=$G timeout -k 10 400 python -u bench.py $C4 --json-out $O/c4_g$G.json > $O/c4_g$G.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
  echo "c4 adamw_grid=$G: $(python -c "import json;j=json.load(open('$O/c4_g$G.json'));print(j['ms_per_step'],j['value'])")"
done
echo done
