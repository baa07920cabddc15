#!/bin/bash
# round 4 pass AI: PMC counters of the attention backward key-block kernel, old (17) vs new (273)
# end-of-tile wait: MFMA busy cycles, wave cycles and wait cycles per dispatch
OUT=gpurun_out/r4ai; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for P in 17 273; do
  MXLLM_ATTN_BWD8_PRIO=$P timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
     --output-format csv -d $ROOT/$OUT/pmc_$P -o run -- python3 $ROOT/bench/attn_bench.py 2 64 8 2048 128 lite > $ROOT/$OUT/pmc_$P.log 2>&1 || { echo "pmc $P rc=$?"; tail -3 $ROOT/$OUT/pmc_$P.log; exit 1; }
  ls $ROOT/$OUT/pmc_$P
done
