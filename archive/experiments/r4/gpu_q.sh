#!/bin/bash
# round 4 pass Q: config-4 proxy with the MLP activation recomputed in the un-checkpointed layers
# (m = swiglu(gu) not saved): HBM and step time at 40 / 32 / 24 checkpointed layers
OUT=gpurun_out/r4q; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k "recompute or train_step" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
for CK in 40 32 24; do
  C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers $CK --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
  timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/c4_ck$CK.json > $OUT/c4_ck$CK.log 2>&1 || { echo "c4 ck$CK rc=$?"; tail -3 $OUT/c4_ck$CK.log; exit 1; }
  echo "c4 ck$CK: $(python -c "import json;j=json.load(open('$OUT/c4_ck$CK.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])")"
done
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 40 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
MXLLM_RECOMPUTE_SWIGLU=0 timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/c4_ck40_saved.json > $OUT/c4_ck40_saved.log 2>&1 || { echo "c4 saved rc=$?"; exit 1; }
echo "c4 ck40 saved m: $(python -c "import json;j=json.load(open('$OUT/c4_ck40_saved.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])")"
