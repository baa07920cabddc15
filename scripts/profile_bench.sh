#!/bin/bash
# Kernel-level profile of the headline bench (run on the GPU box via gpurun).
# usage: scripts/profile_bench.sh <outname> [bench args...]
set -e
NAME=${1:-prof}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py "$@" > $OUT/bench.log 2>&1
