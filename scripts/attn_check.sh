#!/bin/bash
# Attention kernels on the GPU: numerics (incl. the 70B training shape) then the microbenchmark.
# usage: scripts/attn_check.sh <tag>   (outputs gpurun_out/<tag>/)
set -e
TAG=${1:-attn}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $OUT/tests.log 2>&1
timeout -k 10 120 python bench/attn_bench.py > $OUT/bench.json 2> $OUT/bench.err
