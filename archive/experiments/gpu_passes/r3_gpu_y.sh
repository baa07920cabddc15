#!/bin/bash
# Round-3 GPU pass Y: is the GPU crash + resume deterministic?  (a) two resumes from the same step-150
# checkpoint; (b) the uninterrupted vs crash + resume pair with the overlapped AdamW off.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3y
mkdir -p $O
rm -rf /tmp/fy*
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 10 --lr 2e-5 --warmup-steps 20 --steps 200"
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB --save-every 100 \
  --fault-rank 0 --fault-step 105 --fault-kind raise --metrics-file $O/p1.jsonl > $O/p1.log 2>&1 || true
cp -r /tmp/fyB /tmp/fyC
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB --save-every 100000 --metrics-file $O/r1.jsonl > $O/r1.log 2>&1
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyC --save-every 100000 --metrics-file $O/r2.jsonl > $O/r2.log 2>&1
python scripts/compare_resume.py $O/r1.jsonl $O/p1.jsonl $O/r2.jsonl > $O/resume_vs_resume.txt 2>&1 || true
export MXLLM_OVERLAP_ADAMW=0
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyA0 --save-every 100000 --metrics-file $O/full0.jsonl > $O/full0.log 2>&1
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB0 --save-every 100 \
  --fault-rank 0 --fault-step 105 --fault-kind raise --metrics-file $O/p10.jsonl > $O/p10.log 2>&1 || true
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB0 --save-every 100000 --metrics-file $O/p20.jsonl > $O/p20.log 2>&1
python scripts/compare_resume.py $O/full0.jsonl $O/p10.jsonl $O/p20.jsonl > $O/no_overlap.txt 2>&1 || true
