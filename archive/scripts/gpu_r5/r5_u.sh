#!/bin/bash
# Round-5 GPU pass U: fused clip-norm coverage on an 8B-shaped model (diagnostic)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5u
mkdir -p $O
timeout -k 10 300 python -u scripts/diag/fused_norm_coverage.py > $O/coverage.txt 2>&1 || { echo "rc=$?"; tail -20 $O/coverage.txt; exit 1; }
cat $O/coverage.txt
