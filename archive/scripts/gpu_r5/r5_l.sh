#!/bin/bash
# Round-5 GPU pass L: attention backward straight into d(qkv) (attn_bwd_rope) + vectorised adapter
# copy: parity, the attention / model / train GPU suites, headline and config-2 A/B vs MXLLM_ATTN_DQ_ROPE=0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5l
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_attn_dqkv_gpu.py tests/test_copy2d_gpu.py > $O/new_tests.log 2>&1
rc=$?; tail -2 $O/new_tests.log; [ $rc -eq 0 ] || { echo "new tests failed rc=$rc"; grep -E "^E " $O/new_tests.log | head -20; exit 1; }
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py tests/test_fused_epi_gpu.py tests/test_strict_parity_gpu.py tests/test_determinism_gpu.py > $O/suites.log 2>&1
rc=$?; tail -2 $O/suites.log; [ $rc -eq 0 ] || { echo "suites rc=$rc"; grep -E "FAILED|^E " $O/suites.log | head -20; exit 1; }
for i in 1 2; do
  for F in 0 1; do
    MXLLM_ATTN_DQ_ROPE=$F timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-calibrate --json-out $O/bench_dqrope${F}_$i.json > $O/bench_dqrope${F}_$i.log 2>&1 || { echo "bench rc=$?"; exit 1; }
    echo "dq_rope=$F run $i: $(python -c "import json;j=json.load(open('$O/bench_dqrope${F}_$i.json'));c=j['config2_8b_full'];print(j['value'],j['ms_per_step'],j['final_loss'],'| c2',c['value'],c['ms_per_step'])")"
  done
done
echo done
