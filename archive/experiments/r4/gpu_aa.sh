#!/bin/bash
# round 4 pass AA: re-tune hipBLASLt / rocBLAS solutions for the headline's library GEMMs (the
# gate-up forward shape has no table entry), then a same-box A/B of the old vs merged table
OUT=gpurun_out/r4aa; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench/tune_headline.py --out $OUT/merged.csv --max-ms 200 --steps 2 --warmup 1 > $OUT/tune.log 2>&1 || { echo "tune rc=$?"; tail -5 $OUT/tune.log; exit 1; }
tail -2 $OUT/tune.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --config2 off --no-calibrate > $OUT/bench_old_$i.json 2> $OUT/bench_old_$i.err || { echo "old rc=$?"; exit 1; }
  MXLLM_GEMM_TABLE=$OUT/merged.csv timeout -k 10 400 python bench.py --config2 off --no-calibrate > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "new rc=$?"; exit 1; }
  echo "run $i: old $(python -c "import json;print(json.load(open('$OUT/bench_old_$i.json'))['ms_per_step'])") new $(python -c "import json;print(json.load(open('$OUT/bench_new_$i.json'))['ms_per_step'])")"
done
