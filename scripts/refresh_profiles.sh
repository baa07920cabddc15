#!/bin/bash
# Headline numbers + rocprof evidence in one GPU call (run via gpurun).
#   1. unprofiled 70B LoRA bench (the number we quote)
#   2. rocprofv3 --kernel-trace --stats of a short run (per-kernel time)
#   3. rocprofv3 --marker-trace --kernel-trace (roctx phase ranges from the native library)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-refresh}
mkdir -p $OUT
cd $ROOT
timeout -k 10 480 python3 bench.py --steps 6 --warmup 2 --json-out $OUT/bench70b.json > $OUT/bench70b.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 > $OUT/stats.log 2>&1
timeout -k 10 480 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $OUT/markers -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 > $OUT/markers.log 2>&1
