#!/bin/bash
# 70B LoRA step with the committed GEMM table vs the round-1 table (same box).
set -e
git_old=${1:?path to the older table (e.g. git show HEAD~1:mxllm/tuning/tunableop_gfx950.csv > old.csv)}
timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2q_new_table.json 2>/dev/null
MXLLM_GEMM_TABLE=$git_old timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2q_old_table.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2q_new_table2.json 2>/dev/null
