#!/bin/bash
# Round-3 GPU pass J: overlapped AdamW scheduling on the 8B full fine-tune (config 2):
# step on a high-priority stream / AdamW on the lowest (MXLLM_STEP_PRIORITY=1) and
# uncapped AdamW grid (short-lived workgroups), A/B with the defaults; bitwise overlap
# test under the priority streams.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3j
mkdir -p $O
MXLLM_STEP_PRIORITY=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "overlapped or bench" > $O/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "embedding or transpose" tests/test_train_gpu.py tests/test_model_gpu.py > $O/tests2.log 2>&1
B="python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --config2 off --config3 off --config4 off"
for r in 1 2; do
  timeout -k 10 200 $B --json-out $O/8b_base_$r.json > $O/8b_base_$r.log 2>&1
  MXLLM_STEP_PRIORITY=1 timeout -k 10 200 $B --json-out $O/8b_prio_$r.json > $O/8b_prio_$r.log 2>&1
  MXLLM_ADAMW_GRID=1000000000 timeout -k 10 200 $B --json-out $O/8b_grid_$r.json > $O/8b_grid_$r.log 2>&1
  MXLLM_STEP_PRIORITY=1 MXLLM_ADAMW_GRID=1000000000 timeout -k 10 200 $B --json-out $O/8b_both_$r.json > $O/8b_both_$r.log 2>&1
done
