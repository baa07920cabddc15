#!/bin/bash
# Round-5 GPU pass G: attention forward two-group ping-pong kernel (MXLLM_ATTN_FWD=pp): parity, then
# timing against the default (alternating), and the 70B LoRA headline A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5g
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
MXLLM_ATTN_FWD=pp timeout -k 10 400 $T tests/test_kernels_gpu.py -k "attn or attention" tests/test_strict_parity_gpu.py -k "attention" > $O/pp_tests.log 2>&1 || { echo "pp parity failed"; tail -5 $O/pp_tests.log; exit 1; }
tail -1 $O/pp_tests.log
for i in 1 2; do
  for RG in def pp; do
    V=${RG/def/}
    MXLLM_ATTN_FWD=$V timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/b2_${RG}_$i.txt 2>&1 || { echo "bench failed"; exit 1; }
    MXLLM_ATTN_FWD=$V timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $O/b16_${RG}_$i.txt 2>&1 || { echo "bench16 failed"; exit 1; }
    MXLLM_ATTN_FWD=$V timeout -k 10 120 python -u bench/attn_bench.py 1 32 8 8192 128 lite > $O/s8k_${RG}_$i.txt 2>&1 || { echo "bench8k failed"; exit 1; }
    echo "$RG $i: $(tail -1 $O/b2_${RG}_$i.txt | cut -c1-90) | $(tail -1 $O/b16_${RG}_$i.txt | cut -c1-90) | $(tail -1 $O/s8k_${RG}_$i.txt | cut -c1-90)"
  done
done
echo done
