#!/bin/bash
# Round-3 GPU pass AA: where the remaining run-to-run variation comes from -- two from-scratch 1B
# fine-tunes with hipBLASLt (default) and two with rocBLAS (TORCH_BLAS_PREFER_HIPBLASLT=0).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3aa
mkdir -p $O
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 10 --lr 2e-5 --warmup-steps 20 --steps 200"
for i in 1 2; do
  timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --metrics-file $O/blaslt$i.jsonl > $O/blaslt$i.log 2>&1
done
for i in 1 2; do
  TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --metrics-file $O/rocblas$i.jsonl > $O/rocblas$i.log 2>&1
done
python scripts/compare_resume.py $O/blaslt1.jsonl $O/blaslt2.jsonl $O/blaslt2.jsonl > $O/blaslt_pair.txt 2>&1 || true
python scripts/compare_resume.py $O/rocblas1.jsonl $O/rocblas2.jsonl $O/rocblas2.jsonl > $O/rocblas_pair.txt 2>&1 || true
