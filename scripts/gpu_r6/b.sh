#!/bin/bash
# r6 pass B: light-schedule kernels with 4-deep memory-level parallelism: exactness, then the contention probe.
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_multirank_gpu.py::test_peer_collectives_exact_on_shared_gpu" > gpurun_out/r6b/tests.log 2>&1 \
  || { tail -40 gpurun_out/r6b/tests.log; exit 1; }
tail -6 gpurun_out/r6b/tests.log
timeout -k 10 600 python -u bench/comm_contention_probe.py --mb 256 --reps 20 --gemms 60 --light-mb 128 \
  --configs light:8,light:16,light:32,light:64,light:16:bf16,light:32:bf16 \
  2> gpurun_out/r6b/contention.err | tee gpurun_out/r6b/contention.jsonl
