#!/bin/bash
# round 4: long context on one MI355X: 8B full fine-tune at S = 8k / 16k / 32k
# (micro-batch 1, activation checkpointing, chunked LM-head CE) + attention TF/s at those lengths
OUT=gpurun_out/r4_long; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for S in 8192 16384 32768; do
  timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt \
     --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S$S.json > $OUT/8b_full_S$S.log 2>&1
  rc=$?; echo "S=$S rc=$rc: $(cut -c1-300 $OUT/8b_full_S$S.json 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
for S in 2048 8192 16384 32768; do
  timeout -k 10 120 python -u bench/attn_bench.py 1 64 8 $S 128 lite > $OUT/attn_70b_S$S.json 2>&1 || exit $?
  timeout -k 10 120 python -u bench/attn_bench.py 1 32 8 $S 128 lite > $OUT/attn_8b_S$S.json 2>&1 || exit $?
  echo "attn S=$S: $(tail -1 $OUT/attn_70b_S$S.json)"
done
