#!/bin/bash
# r6 pass J: LoRA qkv with RoPE fused into its tail-balanced GEMM -- parity, then a same-box headline A/B
set -o pipefail
OUT=gpurun_out/r6j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_epi_gpu.py tests/test_model_gpu.py -k "rope or lora" > $OUT/tests.log 2>&1 \
  || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for run in 1 0 1 0; do
  tag=qr${run}_$((++i))
  MXLLM_LORA_QKV_ROPE=$run timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --config2 off --no-calibrate --json-out $OUT/head_$tag.json > $OUT/head_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 $OUT/head_$tag.log; exit 1; }
  echo "$tag: $(python -c "import json;j=json.load(open('$OUT/head_$tag.json'));print(j['value'],j['ms_per_step'],j['gpu_after_timed_steps'])")"
done
