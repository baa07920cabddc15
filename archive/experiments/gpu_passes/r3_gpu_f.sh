#!/bin/bash
# Round-3 GPU pass F: LDS-staged lora_xwt (numerics + in-process A/B), then the
# GEMM-table A/B of pass E2 (70B LoRA headline, committed vs re-tuned table).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lora" --timeout 120 --timeout-method thread > $O/lora_tests.log 2>&1
timeout -k 10 300 python -u bench/lora_xwt_ab.py > $O/xwt_ab.log 2>&1
for t in old new old2 new2; do
  if [ $t = new ] || [ $t = new2 ]; then export MXLLM_GEMM_TABLE=$ROOT/mxllm/tuning/candidate.csv; else unset MXLLM_GEMM_TABLE; fi
  timeout -k 10 300 python bench.py --steps 12 --warmup 4 --config2 off --config3 off --config4 off --json-out $O/70b_$t.json > $O/70b_$t.log 2>&1
done
