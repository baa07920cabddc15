#!/bin/bash
# round 4 pass F: deterministic mode (MXLLM_DETERMINISTIC=1, every GEMM on gemm8) -- a 300-step 1B full
# fine-tune uninterrupted vs crashed at step 160 + resumed from its step-150 checkpoint, every step
# logged, final-weight digests; then the mode's cost on the headline (same box, default vs deterministic)
OUT=gpurun_out/r4f; mkdir -p $OUT
export PYTHONUNBUFFERED=1 MXLLM_DETERMINISTIC=1
rm -rf /tmp/dtA /tmp/dtB
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 1 --lr 2e-5 --warmup-steps 20 --steps 300"
timeout -k 10 400 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtA --save-every 100000 --metrics-file $OUT/full.jsonl > $OUT/full.log 2>&1 || { echo "full rc=$?"; exit 1; }
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtB --save-every 150 \
  --fault-rank 0 --fault-step 160 --fault-kind raise --metrics-file $OUT/part1.jsonl > $OUT/part1.log 2>&1
echo "part1 rc=$? (the injected fault's, by design)"
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtB --save-every 100000 --metrics-file $OUT/part2.jsonl > $OUT/part2.log 2>&1 || { echo "part2 rc=$?"; exit 1; }
python scripts/compare_resume.py $OUT/full.jsonl $OUT/part1.jsonl $OUT/part2.jsonl > $OUT/compare.txt 2>&1; tail -2 $OUT/compare.txt
rm -rf /tmp/dtA /tmp/dtB
unset MXLLM_DETERMINISTIC
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/bench_default_$i.json 2>/dev/null || exit 1
  MXLLM_DETERMINISTIC=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/bench_det_$i.json 2>/dev/null || exit 1
  echo "default $i: $(python -c "import json;j=json.load(open('$OUT/bench_default_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")  deterministic $i: $(python -c "import json;j=json.load(open('$OUT/bench_det_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")"
done
