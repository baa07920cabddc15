#!/bin/bash
# round 4 pass AC: attention at the 70B training shape -- all dQ modes, and the forward's phase profile
OUT=gpurun_out/r4ac; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u bench/attn_bench.py 2 64 8 2048 128 > $OUT/attn_modes.txt 2>&1 || { echo "rc=$?"; tail -3 $OUT/attn_modes.txt; exit 1; }
grep shape $OUT/attn_modes.txt
MXLLM_ATTN_PROF=1 timeout -k 10 200 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/attn_prof.txt 2>&1 || { echo "prof rc=$?"; tail -3 $OUT/attn_prof.txt; exit 1; }
grep -v "^{" $OUT/attn_prof.txt | tail -20
