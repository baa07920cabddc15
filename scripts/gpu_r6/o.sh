#!/bin/bash
# r6 pass O: re-tune the hipBLASLt/rocBLAS selection for every GEMM of the headline step (TunableOp,
# merged with the committed table: faster of the two per shape), then a same-box headline A/B of the
# merged table vs the committed one (interleaved, config 2 off)
OUT=gpurun_out/r6o; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench/tune_headline.py --out $OUT/merged.csv --steps 2 --warmup 1 > $OUT/tune.log 2>&1 || { echo "tune rc=$?"; tail -20 $OUT/tune.log; exit 1; }
tail -2 $OUT/tune.log
for i in 1 2; do
  MXLLM_GEMM_TABLE=$OUT/merged.csv timeout -k 10 400 python bench.py --config2 off > $OUT/head_new_$i.json 2> $OUT/head_new_$i.err || { echo "bench rc=$?"; tail -5 $OUT/head_new_$i.err; exit 1; }
  echo "new table run $i: $(python -c "import json;j=json.load(open('$OUT/head_new_$i.json'));print(j['value'],j['ms_per_step'])")"
  timeout -k 10 400 python bench.py --config2 off > $OUT/head_old_$i.json 2> $OUT/head_old_$i.err || { echo "bench rc=$?"; tail -5 $OUT/head_old_$i.err; exit 1; }
  echo "committed table run $i: $(python -c "import json;j=json.load(open('$OUT/head_old_$i.json'));print(j['value'],j['ms_per_step'])")"
done
echo done
