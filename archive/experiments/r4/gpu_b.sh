#!/bin/bash
# round 4 pass B: gemm8 numerics + new GPU tests + shape probe, then the r2-vs-HEAD A/B
OUT=gpurun_out/r4b; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm8_gpu.py tests/test_kernels_gpu.py::test_chunked_lm_head_ce_matches_unchunked_gpu "tests/test_train_gpu.py::test_zero3_overlapped_adamw_bitwise_gpu" tests/test_train_gpu.py::test_zero3_emulated_world4_one_step_gpu tests/test_train_gpu.py::test_zero3_matches_ddp_per_parameter_gpu -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -15 $OUT/tests.txt; echo "tests rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
if grep -q "test_gemm8_orders.*PASSED" $OUT/tests.txt; then
  timeout -k 10 400 python -u bench/gemm8_probe.py --json-out $OUT/probe.json > $OUT/probe.txt 2>&1
  rc=$?; tail -3 $OUT/probe.txt; echo "probe rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
fi
bash experiments/r4/ab_r2_head.sh
