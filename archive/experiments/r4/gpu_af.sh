#!/bin/bash
# round 4 pass AF: attention backward phase cycles with the counted end-of-tile wait (default 273)
OUT=gpurun_out/r4af; mkdir -p $OUT
export PYTHONUNBUFFERED=1
MXLLM_ATTN_PROF=1 timeout -k 10 200 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/attn_prof.txt 2>&1 || { echo "prof rc=$?"; tail -3 $OUT/attn_prof.txt; exit 1; }
grep -v "^{" $OUT/attn_prof.txt | tail -4
