#!/bin/bash
# Round-3 GPU pass U: attention backward DMA issue schedule (MXLLM_ATTN_BWD8_PRIO 17 vs 145 = early
# spread) -- numerics tests with the new schedule, alternating-process microbenchmarks, phase profile.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3u
mkdir -p $O
MXLLM_ATTN_BWD8_PRIO=209 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for p in 17 145 81 209; do
    for b in 2 16; do
      MXLLM_ATTN_BWD8_PRIO=$p timeout -k 10 120 python -u bench/attn_bench.py $b 64 8 2048 128 \
        | sed "s/^/{\"prio\": $p, \"round\": $i, \"r\": /; s/$/}/" >> $O/ab.jsonl
    done
  done
done
MXLLM_ATTN_BWD8_PRIO=209 MXLLM_ATTN_PROF=1 timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 > $O/prof_b2_209.log 2>&1
