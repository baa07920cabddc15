#!/bin/bash
# Round-3 GPU pass I: gradient-norm partials per DDP bucket on a side stream during the
# backward -- GPU tests, then the 8B full fine-tune (BASELINE config 2) A/B.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py > $O/tests.log 2>&1
B="python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --config2 off --config3 off --config4 off"
for r in 1 2; do
  for v in 1 0; do
    MXLLM_NORM_OVERLAP=$v timeout -k 10 200 $B --json-out $O/8b_norm${v}_$r.json > $O/8b_norm${v}_$r.log 2>&1
  done
done
