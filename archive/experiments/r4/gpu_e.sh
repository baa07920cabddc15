#!/bin/bash
# round 4 pass E: gemm8 ablations (barrier / MFMA-per-barrier share), then re-probe with the
# permlane16 bf16 epilogue (nn / tt forms) and rewrite the win table
OUT=gpurun_out/r4e; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_gemm8_gpu.py -q --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 200 python -u bench/gemm8_probe.py --ablate --layout-exp-only --rounds 5 > $OUT/ablate.txt 2>&1 || { echo "ablate rc=$?"; exit 1; }
grep ablate $OUT/ablate.txt
STAMPS_JSON=$OUT/stamps.json timeout -k 10 120 python -u bench/gemm8_stamps.py 8 4 > $OUT/stamps.txt 2>&1 || { echo "stamps rc=$?"; exit 1; }
cat $OUT/stamps.txt
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_gfx950.json
timeout -k 10 600 python -u bench/gemm8_probe.py --aug --ph4 --forms nn,tt,tt32,tn --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe.json > $OUT/probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
tail -1 $OUT/probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/suite.txt 2>&1
rc=$?; tail -4 $OUT/suite.txt; echo "gpu suite rc=$rc"
