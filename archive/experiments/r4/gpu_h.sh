#!/bin/bash
# round 4 pass H: SwiGLU fused with the LoRA tails (csrc/kernels/lora.hip swiglu_lora_kernel):
# numerics, model-level equivalence, speed vs the unfused pair (column-split sweep), headline A/B
OUT=gpurun_out/r4h; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "gpu suite rc=$rc"; exit 1; }
timeout -k 10 300 python -u bench/swiglu_lora_probe.py --cs 0,1,2,4 --rounds 5 --json-out $OUT/probe.json > $OUT/probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
cut -c1-400 $OUT/probe.txt
timeout -k 10 300 python -u bench/lora_probe.py --wgs 256,512,1024,2048 --rounds 3 --json-out $OUT/lora_probe.json > $OUT/lora_probe.txt 2>&1 || { echo "lora probe rc=$?"; exit 1; }
cut -c1-300 $OUT/lora_probe.txt
for i in 1 2; do
  MXLLM_SWIGLU_LORA=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2 off --config2-mb4 off --no-calibrate > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "off $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'])")  on $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'])")"
done
