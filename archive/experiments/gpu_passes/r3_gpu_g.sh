#!/bin/bash
# Round-3 GPU pass G: in-launch decode split merge (hand-off protocols) — numerics, engine
# tests, 8B serve A/B vs the combine kernel; lora_xwt in-launch split reduction A/B;
# LDS-staged lora_xwt A/B on the 70B headline.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u bench/decode_handoff_stress.py > $O/handoff_stress.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_kvcache.py tests/test_serve.py tests/test_sampling.py > $O/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k lora > $O/lora_tests.log 2>&1
timeout -k 10 300 python -u bench/lora_xwt_ab.py > $O/xwt_ab2.log 2>&1
for r in 1 2; do
  for v in fused kernel; do
    MXLLM_DECODE_COMBINE=$v timeout -k 10 300 python bench/serve_bench.py --model llama3.1-8b --batches 1,4,64 --requests 0 --json-out $O/serve8b_${v}_$r.json > $O/serve8b_${v}_$r.log 2>&1
  done
done
for r in 1 2; do
  for v in 1 0; do
    MXLLM_DECODE_PREFETCH=$v timeout -k 10 300 python bench/serve_bench.py --model llama3.1-8b --batches 1,4 --requests 0 --json-out $O/serve8b_pf${v}_$r.json > $O/serve8b_pf${v}_$r.log 2>&1
  done
done
for r in 1 2; do
  for v in lds reg; do
    MXLLM_LORA_XWT=$v timeout -k 10 300 python bench.py --steps 12 --warmup 4 --config2 off --config3 off --config4 off --json-out $O/70b_xwt_${v}_$r.json > $O/70b_xwt_${v}_$r.log 2>&1
  done
done
