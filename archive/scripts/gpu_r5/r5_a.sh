#!/bin/bash
# Round-5 GPU pass A: peer-memory multi-rank tests, strict parity, fused epilogues, config-2 A/B.
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 300 $T tests/test_fused_epi_gpu.py tests/test_gemm8_gpu.py > $O/fused.log 2>&1 || { echo "fused tests failed"; exit 1; }
timeout -k 10 600 $T tests/test_multirank_gpu.py tests/test_comm.py > $O/mr.log 2>&1 || { echo "multirank failed"; exit 1; }
timeout -k 10 400 $T tests/test_strict_parity_gpu.py > $O/strict.log 2>&1 || echo "strict parity failed (continuing)"
for f in 1 0; do
  MXLLM_FUSED_EPI=$f timeout -k 10 240 python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 \
    --no-calibrate --config2 off --json-out $O/c2_fused$f.json > $O/c2_fused$f.log 2>&1 || { echo "bench fused=$f failed"; exit 1; }
done

# attention forward ring depth: parity at ring 3 / 4, then timing (B2 / B16, 70B heads)
for RG in 3 4; do
  MXLLM_ATTN_FWD_RING=$RG timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" tests/test_strict_parity_gpu.py -k "attention" > $O/attn_ring$RG.log 2>&1 || echo "ring $RG parity FAILED"
done
# staggered attention backward (MXLLM_ATTN_BWD8=2): parity first, then timing beside the default
MXLLM_ATTN_BWD8=2 timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" tests/test_strict_parity_gpu.py -k "attention" > $O/attn_bwd_stag.log 2>&1 && STAG_OK=1 || { echo "bwd stagger parity FAILED"; STAG_OK=0; }
if [ "$STAG_OK" = 1 ]; then
  for i in 1 2; do
    for BW in 1 2; do
      MXLLM_ATTN_BWD8=$BW timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/bwd_b2_bw${BW}_$i.txt 2>&1 || { echo "bwd bench failed"; exit 1; }
      MXLLM_ATTN_BWD8=$BW timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $O/bwd_b16_bw${BW}_$i.txt 2>&1 || { echo "bwd bench16 failed"; exit 1; }
    done
  done
fi
for i in 1 2; do
  for RG in 0 3 4; do
    MXLLM_ATTN_FWD_RING=$RG timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/ab2_r${RG}_$i.txt 2>&1 || { echo "attn bench ring $RG failed"; exit 1; }
    MXLLM_ATTN_FWD_RING=$RG timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $O/ab16_r${RG}_$i.txt 2>&1 || { echo "attn bench16 ring $RG failed"; exit 1; }
  done
done
echo done2
