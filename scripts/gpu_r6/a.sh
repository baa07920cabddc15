#!/bin/bash
# r6 pass A: peer collectives (light + resident schedules), multi-rank trainers on the light default,
# then the collective / GEMM contention probe (profiles/r6a/).
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_multirank_gpu.py > gpurun_out/r6a/tests.log 2>&1 || { tail -40 gpurun_out/r6a/tests.log; exit 1; }
tail -15 gpurun_out/r6a/tests.log
timeout -k 10 400 python -u bench/comm_contention_probe.py --mb 256 --reps 20 --gemms 60 \
  --configs resident:32,resident:64,light:32,light:64,light:128,light:256,light:128:bf16 \
  > gpurun_out/r6a/contention.jsonl 2> gpurun_out/r6a/contention.err || { tail -30 gpurun_out/r6a/contention.err; exit 1; }
cat gpurun_out/r6a/contention.jsonl
