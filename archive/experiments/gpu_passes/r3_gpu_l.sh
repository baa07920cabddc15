#!/bin/bash
# Round-3 GPU pass L: CU-masked / lagged overlapped AdamW on the 8B full fine-tune step.
#  1. bench/cu_mask_probe.hip: where a CU-masked stream runs (XCC / CU ids) and the HBM
#     bandwidth an AdamW-shaped stream reaches on each CU subset
#  2. the whole GPU suite at this tree (includes the bitwise schedule tests)
#  3. bench/adamw_overlap_ab.py: schedule variants, interleaved rounds, one process
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3l
mkdir -p $O build
hipcc -O3 --offload-arch=gfx950 bench/cu_mask_probe.hip -o build/cu_mask_probe
timeout -k 10 120 ./build/cu_mask_probe > $O/cu_mask_probe.jsonl 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 900 python -u bench/adamw_overlap_ab.py --rounds 2 --json-out $O/ab.jsonl \
  base= lag1=MXLLM_ADAMW_LAG=1 lag3=MXLLM_ADAMW_LAG=3 cu32=MXLLM_ADAMW_CUS=mod8:1 cu64=MXLLM_ADAMW_CUS=mod8:2 \
  cu96=MXLLM_ADAMW_CUS=mod8:3 cu64lag3=MXLLM_ADAMW_CUS=mod8:2,MXLLM_ADAMW_LAG=3 > $O/ab.log 2>&1
