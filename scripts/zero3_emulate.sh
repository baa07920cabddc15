#!/bin/bash
# BASELINE config 4 sizing proxy on ONE GPU: Llama-3.1-70B full fine-tune, ZeRO-3 with
# world-8 shard sizes (gathers tile the local shard; no link traffic), 80 layers.
# usage: scripts/zero3_emulate.sh <tag> [extra bench args]   (outputs gpurun_out/<tag>/)
set -e
TAG=${1:-z3emu}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for cfg in "--act-ckpt --micro-batch 2" "--act-ckpt --micro-batch 4" "--micro-batch 2"; do
  name=$(echo $cfg | tr -d ' -')
  timeout -k 10 420 python bench.py --model llama3.1-70b --finetune full --parallel zero3 --emulate-world 8 \
      $cfg --steps 3 --warmup 1 "$@" > $OUT/$name.json 2> $OUT/$name.err
done
