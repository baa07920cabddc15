#!/bin/bash
# Round-2 evidence runs: host-sync audit of the 8B full step; kernel profile of the 70B ZeRO-3
# world-8 emulation (config-4 per-rank proxy).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash $ROOT/scripts/trace_syncs.sh r2m_syncs_8b --model llama3.1-8b --finetune full --steps 3 --warmup 2
bash $ROOT/scripts/profile_bench.sh r2m_prof_z3emu --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --micro-batch 4 --emulate-world 8 --steps 2 --warmup 1
