#!/bin/bash
# round 4 pass B: gemm8 numerics + shape probe, then the r2-vs-HEAD A/B
OUT=gpurun_out/r4b; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -m pytest tests/test_gemm8_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -5 $OUT/tests.txt; echo "gemm8 tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python -u bench/gemm8_probe.py --json-out $OUT/probe.json > $OUT/probe.txt 2>&1
  rc=$?; tail -3 $OUT/probe.txt; echo "probe rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
fi
bash experiments/r4/ab_r2_head.sh
