#!/bin/bash
# round 4 pass F: (1) fp32 dW at T 8192 (config-4 shapes) with the 4-phase schedule -> table;
# (2) same-box A/B of the bench line with / without gemm8 (new table); (3) config-4 proxy;
# (4) deterministic mode: 300-step 1B crash + resume vs uninterrupted, and its headline cost
OUT=gpurun_out/r4f; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_gfx950.json
timeout -k 10 300 python -u bench/gemm8_probe.py --model 70b --tokens 8192 --forms tt32 --ph4 --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_t8192.json > $OUT/probe_t8192.txt 2>&1 || { echo "probe8k rc=$?"; exit 1; }
tail -1 $OUT/probe_t8192.txt
cp $OUT/gemm8_gfx950.json mxllm/tuning/gemm8_gfx950.json
for i in 1 2; do
  MXLLM_GEMM8=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "off $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'],j['config2_8b_full_mb4']['ms_per_step'])")  on $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'],j['config2_8b_full_mb4']['ms_per_step'],j['calibration'])")"
done
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
timeout -k 10 600 python -u bench.py $C4 --json-out $OUT/c4_on.json > $OUT/c4_on.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
echo "c4: $(python -c "import json;j=json.load(open('$OUT/c4_on.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'])")"
rm -rf /tmp/dtA /tmp/dtB
ARGS="--model llama3.2-1b --finetune full --seq-len 512 --micro-batch 8 --log-every 1 --lr 2e-5 --warmup-steps 20 --steps 300"
export MXLLM_DETERMINISTIC=1
timeout -k 10 400 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtA --save-every 100000 --metrics-file $OUT/full.jsonl > $OUT/full.log 2>&1 || { echo "full rc=$?"; exit 1; }
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtB --save-every 150 \
  --fault-rank 0 --fault-step 160 --fault-kind raise --metrics-file $OUT/part1.jsonl > $OUT/part1.log 2>&1
echo "part1 rc=$? (the injected fault's, by design)"
timeout -k 10 300 python -u src/distributed_finetuning.py $ARGS --ckpt-dir /tmp/dtB --save-every 100000 --metrics-file $OUT/part2.jsonl > $OUT/part2.log 2>&1 || { echo "part2 rc=$?"; exit 1; }
python scripts/compare_resume.py $OUT/full.jsonl $OUT/part1.jsonl $OUT/part2.jsonl > $OUT/compare.txt 2>&1; tail -2 $OUT/compare.txt
rm -rf /tmp/dtA /tmp/dtB
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/bench_det.json 2>/dev/null || exit 1
echo "deterministic: $(python -c "import json;j=json.load(open('$OUT/bench_det.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'],j['config']['gemm'])")"
