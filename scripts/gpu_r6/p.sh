#!/bin/bash
# r6 pass P: PMC counters of the headline's GEMM kernels at the 70B-LoRA shapes (gemm8 4-phase NN / TN,
# hipBLASLt TN): MFMA busy, LDS activity and bank conflicts.  One counter pass (7 SQ + 1 GRBM).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
for c in $C GRBM_GUI_ACTIVE; do grep -q "$c" $O/avail.txt || { echo "counter $c not listed"; exit 1; }; done
MXLLM_GEMM8_PH=4 timeout -s KILL 300 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- \
  python3 $R/bench/gemm8_probe.py --aug-only --rounds 1 --calls 2 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
cd $R
python scripts/pmc_summary.py $O/pmc gemm8_kernel Cijk > $O/summary_raw.txt
head -60 $O/summary_raw.txt
rm -f $(find $O/pmc -name "*counter_collection.csv" -size +20M)
echo done
