#!/bin/bash
# Kernel trace of the graphed 8B decode step at batch 1 (run on the GPU box via gpurun).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-decode_prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $ROOT/bench/serve_bench.py --model llama3.1-8b --batches 64 --decode-steps 32 --requests 4 --new-tokens 4 > $OUT/serve.log 2>&1
