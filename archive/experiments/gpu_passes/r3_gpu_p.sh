#!/bin/bash
# Round-3 GPU pass P: kernel-trace breakdown of the 8B full fine-tune step (BASELINE config 2) at this
# tree, to find the remaining non-HIP (torch) kernels on its critical path.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3p
mkdir -p $O
bash scripts/profile_bench.sh r3p/prof8b --model llama3.1-8b --finetune full --steps 3 --warmup 2
python scripts/step_breakdown.py $O/prof8b/run_kernel_trace.csv 40 > $O/step_breakdown_8b.txt 2>&1 || true
python scripts/overlap_report.py $O/prof8b/run_kernel_trace.csv > $O/overlap_8b.txt 2>&1 || true
