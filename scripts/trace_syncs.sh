#!/bin/bash
# Host-sync audit of the training step: kernel + memory-copy trace (no PMC counters) of a
# short bench run, then list device->host copies inside the last full optimizer step.
# usage: scripts/trace_syncs.sh <tag> [bench args]   (outputs gpurun_out/<tag>/)
set -e
TAG=${1:-syncs}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 $ROOT/bench.py "$@" > $OUT/bench.log 2>&1
python3 $ROOT/scripts/step_copies.py $OUT > $OUT/step_copies.txt
