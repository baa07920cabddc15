#!/bin/bash
# Round-3 GPU pass E2: A/B of the committed GEMM table vs the re-tuned one (mxllm/tuning/candidate.csv: 5 forward shapes re-tuned).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3e
for t in old new old2 new2; do
  if [ $t = new ] || [ $t = new2 ]; then export MXLLM_GEMM_TABLE=$ROOT/mxllm/tuning/candidate.csv; else unset MXLLM_GEMM_TABLE; fi
  timeout -k 10 300 python bench.py --steps 12 --warmup 4 --config2 off --config3 off --config4 off --json-out $O/70b_$t.json > $O/70b_$t.log 2>&1
done
