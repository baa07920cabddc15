#!/bin/bash
# GPU-box validation: kernel/model tests, then the headline bench (and optional extras).
# usage: scripts/gpu_check.sh [tag]    (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-check}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1
timeout -k 10 420 python bench.py --steps 4 --warmup 2 > $OUT/bench70b.log 2>&1
