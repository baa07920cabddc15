#!/bin/bash
# round 4 pass M: tail-balanced gemm8 launch (K-split last wave) for the forward GEMMs whose tile grid
# leaves a short last wave (70B / 70B-LoRA qkv, 8B qkv, LM heads): numerics, probe -> table, A/B
OUT=gpurun_out/r4m; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm8_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "gemm8 tests rc=$rc"; exit 1; }
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_old.json
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_gfx950.json
timeout -k 10 500 python -u bench/gemm8_probe.py --model both --tokens 4096 --forms tn,tt --aug --ph4 --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_tn.json > $OUT/probe_tn.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
grep -E "tail" $OUT/probe_tn.txt | cut -c1-330
tail -1 $OUT/probe_tn.txt
for i in 1 2; do
  cp $OUT/gemm8_old.json mxllm/tuning/gemm8_gfx950.json
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config2-mb4 off --no-calibrate > $OUT/bench_old_$i.json 2> $OUT/bench_old_$i.err || { echo "bench old rc=$?"; exit 1; }
  cp $OUT/gemm8_gfx950.json mxllm/tuning/gemm8_gfx950.json
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --config2-mb4 off --no-calibrate > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "bench new rc=$?"; exit 1; }
  echo "old $i: $(python -c "import json;j=json.load(open('$OUT/bench_old_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")  new $i: $(python -c "import json;j=json.load(open('$OUT/bench_new_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")"
done
