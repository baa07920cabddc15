#!/bin/bash
# Round-3 GPU pass E: re-tune the library GEMM selection for every GEMM of the headline
# (70B LoRA) and of config 2 (8B full, bf16 and fp32-output dW), then A/B both workloads
# with the committed table vs the merged one.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 900 python bench/tune_headline.py --out $O/t1.csv --steps 1 --warmup 1 > $O/tune_70b.log 2>&1
timeout -k 10 600 python bench/tune_headline.py --base $O/t1.csv --out $O/t2.csv --model llama3.1-8b --finetune full --steps 1 --warmup 1 > $O/tune_8b.log 2>&1
timeout -k 10 600 python bench/tune_headline.py --base $O/t2.csv --out $O/t3.csv --model llama3.1-8b --finetune full --grad-dtype fp32 --steps 1 --warmup 1 > $O/tune_8b_fp32.log 2>&1
for t in old new; do
  if [ $t = new ]; then export MXLLM_GEMM_TABLE=$O/t3.csv; fi
  timeout -k 10 400 python bench.py --steps 12 --warmup 4 --config2 off --json-out $O/70b_$t.json > $O/70b_$t.log 2>&1
  timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --json-out $O/8b_$t.json > $O/8b_$t.log 2>&1
done
