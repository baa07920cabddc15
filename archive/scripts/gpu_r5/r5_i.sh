#!/bin/bash
# Round-5 GPU pass I: PMC counters of the default attention forward and backward kernels at the
# 70B training shape (B2 S2048 Hq64 Hkv8 D128): MFMA busy, VALU activity, LDS waits.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA"
for c in $C GRBM_GUI_ACTIVE; do grep -q "$c" $O/avail.txt || { echo "counter $c not listed"; exit 1; }; done
timeout -s KILL 120 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_a -o run -- python3 $R/bench/attn_bench.py 2 64 8 2048 128 lite > $O/pmc_a.log 2>&1 || { echo "pmc a rc=$?"; tail -3 $O/pmc_a.log; exit 1; }
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_SALU"
for c in $C2; do grep -q "$c" $O/avail.txt || { echo "counter $c not listed (pass b skipped)"; echo done; exit 0; }; done
timeout -s KILL 120 rocprofv3 --pmc $C2 GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b -o run -- python3 $R/bench/attn_bench.py 2 64 8 2048 128 lite > $O/pmc_b.log 2>&1 || { echo "pmc b rc=$?"; tail -3 $O/pmc_b.log; exit 1; }
echo done
