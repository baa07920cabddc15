#!/bin/bash
# r6 pass B2: light schedule with non-temporal streams and 8-deep memory parallelism.
set -o pipefail
mkdir -p gpurun_out/r6b2
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_multirank_gpu.py::test_peer_collectives_exact_on_shared_gpu" > gpurun_out/r6b2/tests.log 2>&1 \
  || { tail -40 gpurun_out/r6b2/tests.log; exit 1; }
tail -6 gpurun_out/r6b2/tests.log
timeout -k 10 600 python -u bench/comm_contention_probe.py --mb 256 --reps 20 --gemms 60 --light-mb 128 \
  --configs light:16,light:32,light:64,light:32:bf16,resident:32 \
  2> gpurun_out/r6b2/contention.err | tee gpurun_out/r6b2/contention.jsonl
