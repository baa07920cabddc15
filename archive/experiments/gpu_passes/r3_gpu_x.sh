#!/bin/bash
# Round-3 GPU pass X: lora_xtg with 32-row blocks (two workgroups per CU) -- LoRA kernel tests under
# both block sizes, then the 70B LoRA headline step A/B in one process.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3x
mkdir -p $O
MXLLM_LORA_XTG_ROWS=32 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -q --timeout 120 --timeout-method thread > $O/tests32.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lora" -x -q --timeout 120 --timeout-method thread > $O/tests64.log 2>&1
timeout -k 10 900 python -u bench/adamw_overlap_ab.py --model llama3.1-70b --finetune lora --steps 4 --warmup 2 --rounds 2 --json-out $O/ab.jsonl \
  rows64= rows32=MXLLM_LORA_XTG_ROWS=32 > $O/ab.log 2>&1
