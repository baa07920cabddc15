#!/bin/bash
# Round-3 GPU pass N: packed-fp32 softmax arithmetic in the attention forward (MXLLM_ATTN_FWD_PK)
# -- attention numerics tests, then alternating same-box microbenchmarks (B2 and B16, 70B heads).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3n
mkdir -p $O
MXLLM_ATTN_FWD_PK=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  for pk in 1 0; do
    for b in 2 16; do
      MXLLM_ATTN_FWD_PK=$pk timeout -k 10 120 python -u bench/attn_bench.py $b 64 8 2048 128 \
        | sed "s/^/{\"pk\": $pk, \"round\": $i, \"r\": /; s/$/}/" >> $O/attn_ab.jsonl
    done
  done
done
