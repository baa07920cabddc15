#!/bin/bash
# Round-3 first GPU pass: new training-path GPU tests, the driver bench line (headline +
# config 2), the 8B full fine-tune A/B (optimizer overlap on/off, fp32 gradients) and a
# kernel trace of the overlapped 8B step.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train_gpu.py > $O/tests.log 2>&1
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1
for v in 1 0; do
  MXLLM_OVERLAP_ADAMW=$v timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 \
    --json-out $O/8b_full_ovl$v.json > $O/8b_full_ovl$v.log 2>&1
done
timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --grad-dtype fp32 \
  --json-out $O/8b_full_fp32.json > $O/8b_full_fp32.log 2>&1
bash scripts/profile_bench.sh r3a/prof8b --model llama3.1-8b --finetune full --steps 3 --warmup 2
python scripts/overlap_report.py $O/prof8b/run_kernel_trace.csv > $O/overlap.txt 2>&1
