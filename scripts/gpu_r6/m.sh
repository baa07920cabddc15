#!/bin/bash
# r6 pass M: LoRA overlapped AdamW (per-chunk adapter copies) -- tests, then a same-box headline A/B
# (MXLLM_LORA_OVERLAP_ADAMW 1 vs 0, interleaved, config 2 off)
OUT=gpurun_out/r6m; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_gpu.py > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for v in 1 0; do
    MXLLM_LORA_OVERLAP_ADAMW=$v timeout -k 10 400 python bench.py --config2 off > $OUT/head_ovl${v}_$i.json 2> $OUT/head_ovl${v}_$i.err || { echo "bench rc=$?"; tail -5 $OUT/head_ovl${v}_$i.err; exit 1; }
    echo "ovl=$v run $i: $(python -c "import json;j=json.load(open('$OUT/head_ovl${v}_$i.json'));print(j['value'],j['ms_per_step'])")"
  done
done
echo done
