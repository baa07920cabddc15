#!/bin/bash
# round 4: long context without activation checkpointing where HBM allows (8B full fine-tune,
# micro-batch 1): activations are ~2.6 MB per token over 32 layers, so S 8k / 16k / 32k need
# ~21 / 42 / 84 GB on top of ~112 GB of weights + optimizer state; the attention backward's dS^T
# image is bounded by chunking (mxllm/ops/attention.py attn_bwd)
OUT=gpurun_out/r4_long; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -v --timeout 120 --timeout-method thread > $OUT/tests_attn.txt 2>&1
rc=$?; tail -2 $OUT/tests_attn.txt; [ $rc -eq 0 ] || { echo "attention tests rc=$rc"; exit 1; }
for S in 8192 16384 32768; do
  timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 \
     --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_nockpt.json > $OUT/8b_full_S${S}_nockpt.log 2>&1
  rc=$?; echo "S=$S no ckpt rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_nockpt.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
S=32768
timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt \
   --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_ckpt_bounded.json > $OUT/8b_full_S${S}_ckpt_bounded.log 2>&1
rc=$?; echo "S=$S every layer ckpt rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_ckpt_bounded.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
