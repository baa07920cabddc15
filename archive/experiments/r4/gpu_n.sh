#!/bin/bash
# round 4 pass N: the 70B-LoRA augmented shapes again (incl. the down-projection forward in TN form,
# K = 28672 + 64, never measured before) -> table; headline A/B old vs new table
OUT=gpurun_out/r4n; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_old.json
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_gfx950.json
timeout -k 10 300 python -u bench/gemm8_probe.py --aug-only --ph4 --rounds 5 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_aug.json > $OUT/probe_aug.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
cut -c1-300 $OUT/probe_aug.txt
for i in 1 2; do
  cp $OUT/gemm8_old.json mxllm/tuning/gemm8_gfx950.json
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_old_$i.json 2> $OUT/bench_old_$i.err || { echo "bench old rc=$?"; exit 1; }
  cp $OUT/gemm8_gfx950.json mxllm/tuning/gemm8_gfx950.json
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "bench new rc=$?"; exit 1; }
  echo "old $i: $(python -c "import json;j=json.load(open('$OUT/bench_old_$i.json'));print(j['ms_per_step'])")  new $i: $(python -c "import json;j=json.load(open('$OUT/bench_new_$i.json'));print(j['ms_per_step'])")"
done
