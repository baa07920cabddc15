#!/bin/bash
# Round-3 GPU pass T: phase-cycle profiles (MXLLM_ATTN_PROF=1 diagnostic builds) of the attention
# forward and the 8-wave backward at the 70B training shape, current tree.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3t
mkdir -p $O
MXLLM_ATTN_PROF=1 timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 > $O/prof_b2.log 2>&1
MXLLM_ATTN_PROF=1 timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 > $O/prof_b16.log 2>&1
