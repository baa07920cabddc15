#!/bin/bash
# Round-5 GPU pass B: persistent gemm8 parity + timing vs the one-tile kernel and hipBLASLt.
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gemm8_gpu.py > $O/gemm8_tests.log 2>&1 || { echo "gemm8 tests failed"; exit 1; }
timeout -k 10 420 python -u bench/gemm8_probe.py --model 70b --tokens 4096 --rounds 3 --forms tn,nn,tt32 --aug --ph4 --persist > $O/probe70_t4096.txt 2>&1 || { echo "probe 70b failed"; exit 1; }
timeout -k 10 300 python -u bench/gemm8_probe.py --model 8b --tokens 4096 --rounds 3 --forms tn,nn,tt --ph4 --persist > $O/probe8_t4096.txt 2>&1 || { echo "probe 8b failed"; exit 1; }
echo done
