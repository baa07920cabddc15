#!/bin/bash
# r6 pass G: lora_xtg wave-owns-tile A/B (MXLLM_LORA_XTG_WT) -- parity, then per-projection timing
set -o pipefail
OUT=gpurun_out/r6g; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k lora_grads > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u bench/lora_xtg_wt_ab.py --rounds 6 --calls 20 | tee $OUT/ab_wgs256.jsonl
timeout -k 10 300 python -u bench/lora_xtg_wt_ab.py --rounds 4 --calls 20 --wgs 128 | tee $OUT/ab_wgs128.jsonl
