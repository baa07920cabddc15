#!/bin/bash
# PMC counters for the attention kernels (two passes; counters only, no tracing domains).
# usage: scripts/pmc_attn.sh <tag> [attn_bench args...]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_attn}
shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 $ROOT/bench/attn_bench.py "$@" > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -- python3 $ROOT/bench/attn_bench.py "$@" > $OUT/p2.log 2>&1
python3 $ROOT/scripts/pmc_summary.py $OUT attn_fwd > $OUT/summary_fwd.txt
