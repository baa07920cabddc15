#!/bin/bash
# round 4 pass AB: does the re-tuned gate-up forward entry (rocBLAS 618465) change that GEMM?
OUT=gpurun_out/r4ab; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/tunable_check.py --table experiments/r4/aa_merged_table.csv > $OUT/check_gu.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/check_gu.txt; exit 1; }
timeout -k 10 300 python -u bench/tunable_check.py --table experiments/r4/aa_merged_table.csv --n 8192 --k 28736 > $OUT/check_down.txt 2>&1 || { echo "rc=$?"; exit 1; }
grep shape $OUT/check_gu.txt $OUT/check_down.txt
