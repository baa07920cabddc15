#!/bin/bash
# r6 evidence pass: whole GPU suite, smoke(), the default bench line twice (headline + calibration +
# config 2 / 2-mb4), the config-4 proxy; output under gpurun_out/${FINAL_OUT:-r6_final}.
OUT=gpurun_out/${FINAL_OUT:-r6_final}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 560 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt; grep -E "FAILED|ERROR" $OUT/tests.txt | head -20
[ $rc -le 1 ] || { echo "suite ended abnormally (rc=$rc): stop"; exit 1; }
cp gpurun_out/bench_rehearsal_w*.json $OUT/ 2>/dev/null
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
for i in ${BENCH_RUNS:-1 2}; do
  timeout -k 10 560 python bench.py > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_$i.err; exit 1; }
  echo "bench $i: $(python -c "import json;j=json.load(open('$OUT/bench_$i.json'));print(j['value'],j['ms_per_step'],j['config2_8b_full']['value'],j['config2_8b_full']['ms_per_step'],j['config2_8b_full_mb4']['value'],j['calibration'])")"
done
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/c4_ck0.json > $OUT/c4_ck0.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
echo "c4 ck0: $(python -c "import json;j=json.load(open('$OUT/c4_ck0.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_reserved_gb'])")"
echo done
