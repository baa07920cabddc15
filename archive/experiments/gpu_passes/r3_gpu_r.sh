#!/bin/bash
# Round-3 GPU pass R: PMC counters of the token-major dW kernel forms (70B shapes) -- LDS traffic,
# bank conflicts and MFMA busy, to back the LDS-bound reading in profiles/r3m/README.md.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r3r
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 $ROOT/bench/dw_gemm_probe.py --models 70b --iters 3 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -- python3 $ROOT/bench/dw_gemm_probe.py --models 70b --iters 3 > $OUT/p2.log 2>&1
python3 $ROOT/scripts/pmc_summary.py $OUT dw_gemm Cijk > $OUT/summary.txt
