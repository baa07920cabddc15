#!/bin/bash
# Round-3 GPU pass Z: deterministic tied-embedding backward -- GPU tests, then the crash + resume
# comparison again (pass W) and two resumes from one checkpoint (pass Y part a).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
bash scripts/r3_gpu_w.sh
cp gpurun_out/r3w/compare.txt $O/w_compare.txt
rm -rf /tmp/fy*
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 10 --lr 2e-5 --warmup-steps 20 --steps 200"
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB --save-every 100 \
  --fault-rank 0 --fault-step 105 --fault-kind raise --metrics-file $O/p1.jsonl > $O/p1.log 2>&1 || true
cp -r /tmp/fyB /tmp/fyC
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyB --save-every 100000 --metrics-file $O/r1.jsonl > $O/r1.log 2>&1
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/fyC --save-every 100000 --metrics-file $O/r2.jsonl > $O/r2.log 2>&1
python scripts/compare_resume.py $O/r1.jsonl $O/p1.jsonl $O/r2.jsonl > $O/resume_vs_resume.txt 2>&1 || true
