#!/bin/bash
# Round-3 GPU pass W: fine-tuning convergence + checkpoint/resume on one MI355X with the reference's
# driver (src/distributed_finetuning.py): Llama-3.2-1B full fine-tune on the offline imdb-like reviews,
# 300 steps uninterrupted vs the same run crashed (injected fault) at step 160 and resumed from its
# step-150 checkpoint; the logged losses are compared by scripts/compare_resume.py.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3w
mkdir -p $O
rm -rf /tmp/ftA /tmp/ftB
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 10 --lr 2e-5 --warmup-steps 20"
timeout -k 10 400 python -u src/distributed_finetuning.py $ARGS --steps 300 --ckpt-dir /tmp/ftA --save-every 100000 --metrics-file $O/full.jsonl > $O/full.log 2>&1
# the same 300-step run (same LR schedule), killed by an injected fault at step 160 after the
# step-150 checkpoint; its exit code is the fault's, by design
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --steps 300 --ckpt-dir /tmp/ftB --save-every 150 \
  --fault-rank 0 --fault-step 160 --fault-kind raise --metrics-file $O/part1.jsonl > $O/part1.log 2>&1 || true
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --steps 300 --ckpt-dir /tmp/ftB --save-every 100000 --metrics-file $O/part2.jsonl > $O/part2.log 2>&1
python scripts/compare_resume.py $O/full.jsonl $O/part1.jsonl $O/part2.jsonl > $O/compare.txt 2>&1 || true
