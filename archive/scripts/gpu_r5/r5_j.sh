#!/bin/bash
# Round-5 GPU pass J: collective / GEMM contention on one GPU (two ranks, peer collectives)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/comm_contention_probe.py --mb 256 --reps 20 --gemms 40 --wgs 8,32,64 > $O/contention.txt 2>&1 || { echo "probe failed"; tail -20 $O/contention.txt; exit 1; }
grep peer_wgs $O/contention.txt
echo done
