#!/bin/bash
# round 4 pass Y: fp8 GEMM tests (new dispatch) + kernel profile of the 8B bf16 decode step (batch 1)
OUT=gpurun_out/r4y; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "w8" -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1
rc=$?; tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof8 -o run -- python3 $ROOT/bench/serve_bench.py --model llama3.1-8b --batches 1 --requests 4 --decode-steps 64 > $ROOT/$OUT/prof8.log 2>&1 || { echo "prof rc=$?"; exit 1; }
head -16 $ROOT/$OUT/prof8/run_kernel_stats.csv | cut -c1-160
rm -f $ROOT/$OUT/prof8/run_kernel_trace.csv
