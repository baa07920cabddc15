#!/bin/bash
# Round-5 GPU pass L0: mismatch report of the attn_bwd_rope parity test
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5l0
mkdir -p $O
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_attn_dqkv_gpu.py > $O/t.log 2>&1
grep -E "PASSED|FAILED|differ" $O/t.log | cut -c1-600
echo done
