#!/bin/bash
# Round-3 GPU pass E1: re-tune the library GEMM selection for every GEMM of the headline
# (70B LoRA) and of config 2 (8B full, bf16 and fp32-output dW).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 700 python -u bench/tune_headline.py --out $O/t1.csv --steps 1 --warmup 1 > $O/tune_70b.log 2>&1
timeout -k 10 400 python -u bench/tune_headline.py --base $O/t1.csv --out $O/t2.csv --model llama3.1-8b --finetune full --steps 1 --warmup 1 > $O/tune_8b.log 2>&1
