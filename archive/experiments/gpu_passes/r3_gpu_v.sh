#!/bin/bash
# Round-3 GPU pass V: sharded paths at the final tree -- BASELINE config-4 per-rank proxy (70B full
# ZeRO-3, world-8 shard sizes emulated, 56 of 80 layers checkpointed, micro-batch 4, fp32
# reduce-scatter) and 8B ZeRO-3 vs DDP at world 1.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 500 python -u bench.py --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --json-out $O/z3emu8.json > $O/z3emu8.log 2>&1
timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --parallel zero3 --steps 5 --warmup 2 --json-out $O/z3_8b.json > $O/z3_8b.log 2>&1
timeout -k 10 300 python -u bench.py --model llama3.1-8b --finetune full --parallel zero1 --steps 5 --warmup 2 --json-out $O/z1_8b.json > $O/z1_8b.log 2>&1
