#!/bin/bash
# Round-3 GPU pass B: full GPU suite after the split-master / fresh-gradient changes,
# the 8B full fine-tune A/B (each optimisation switched off in turn), the driver bench
# line and a kernel trace of the 8B step.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
B="python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3"
timeout -k 10 200 $B --json-out $O/8b_default.json > $O/8b_default.log 2>&1
MXLLM_SPLIT_MASTER=0 timeout -k 10 200 $B --json-out $O/8b_nosplit.json > $O/8b_nosplit.log 2>&1
MXLLM_FRESH_GRADS=0 timeout -k 10 200 $B --json-out $O/8b_nofresh.json > $O/8b_nofresh.log 2>&1
MXLLM_OVERLAP_ADAMW=0 timeout -k 10 200 $B --json-out $O/8b_noovl.json > $O/8b_noovl.log 2>&1
MXLLM_ADAMW_GRID=512 timeout -k 10 200 $B --json-out $O/8b_grid512.json > $O/8b_grid512.log 2>&1
timeout -k 10 200 $B --json-out $O/8b_default2.json > $O/8b_default2.log 2>&1
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1
bash scripts/profile_bench.sh r3b/prof8b --model llama3.1-8b --finetune full --steps 3 --warmup 2
python scripts/overlap_report.py $O/prof8b/run_kernel_trace.csv > $O/overlap.txt 2>&1
python scripts/step_breakdown.py $O/prof8b/run_kernel_trace.csv 30 > $O/breakdown.txt 2>&1 || true
