#!/bin/bash
# round 4 pass D: GPU suite (incl. determinism, S=8192 attention, gemm8), o-dX layout experiment,
# long-context 8B fine-tune, config-4 per-rank proxy (overlapped ZeRO-3 AdamW + gemm8 fp32 dW vs off)
OUT=gpurun_out/r4d; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -4 $OUT/tests.txt; echo "gpu suite rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u bench/gemm8_probe.py --layout-exp-only --layout-exp --rounds 3 > $OUT/layout.txt 2>&1 || { echo "layout rc=$?"; exit 1; }
grep layout $OUT/layout.txt | cut -c1-200
bash experiments/r4/long_ctx.sh || { echo "long ctx rc=$?"; exit 1; }
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
timeout -k 10 600 python -u bench.py $C4 --json-out $OUT/c4_on.json > $OUT/c4_on.log 2>&1 || { echo "c4 on rc=$?"; exit 1; }
echo "c4 on: $(python -c "import json;j=json.load(open('$OUT/c4_on.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j.get('zero3'))")"
MXLLM_Z3_ADAMW_OVERLAP=0 MXLLM_GEMM8=0 timeout -k 10 600 python -u bench.py $C4 --json-out $OUT/c4_off.json > $OUT/c4_off.log 2>&1 || { echo "c4 off rc=$?"; exit 1; }
echo "c4 off: $(python -c "import json;j=json.load(open('$OUT/c4_off.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j.get('zero3'))")"
