#!/bin/bash
# Round-5 GPU pass F: strict parity (coverage-test epsilon), attention forward split K/V ring
# (MXLLM_ATTN_FWD_RING=k3) parity + timing + phase cycles against the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5f
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_strict_parity_gpu.py > $O/strict.log 2>&1 || echo "strict parity: failures (see log)"
MXLLM_ATTN_FWD_RING=k3 timeout -k 10 400 $T tests/test_kernels_gpu.py -k "attn or attention" tests/test_strict_parity_gpu.py -k "attention" > $O/k3_tests.log 2>&1 || { echo "k3 parity failed"; tail -5 $O/k3_tests.log; exit 1; }
tail -1 $O/k3_tests.log
for i in 1 2; do
  for RG in def k3; do
    V=${RG/def/}
    MXLLM_ATTN_FWD_RING=$V timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/b2_${RG}_$i.txt 2>&1 || { echo "bench failed"; exit 1; }
    MXLLM_ATTN_FWD_RING=$V timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $O/b16_${RG}_$i.txt 2>&1 || { echo "bench16 failed"; exit 1; }
    echo "$RG $i: $(tail -1 $O/b2_${RG}_$i.txt | cut -c1-120) | $(tail -1 $O/b16_${RG}_$i.txt | cut -c1-120)"
  done
done
for RG in def k3; do
  V=${RG/def/}
  MXLLM_ATTN_PROF=1 MXLLM_ATTN_FWD_RING=$V timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/prof_${RG}.txt 2>&1 || { echo "prof failed"; exit 1; }
  grep -m2 "attn_fwd prof" $O/prof_${RG}.txt || true
done
echo done
