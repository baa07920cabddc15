#!/bin/bash
# round 4 pass J: in-launch (last-arriver) split reduction for the LoRA kernels vs the separate
# reduce launch; attention at the training shape for the record
OUT=gpurun_out/r4j; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/lora_probe.py --rounds 5 --json-out $OUT/lora_probe.json > $OUT/lora_probe.txt 2>&1 || { echo "lora probe rc=$?"; exit 1; }
cut -c1-300 $OUT/lora_probe.txt
timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 > $OUT/attn_b2.txt 2>&1 || { echo "attn rc=$?"; exit 1; }
tail -1 $OUT/attn_b2.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  MXLLM_LORA_FUSED_RED=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "separate $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'])")  fused_red $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'])")"
done
