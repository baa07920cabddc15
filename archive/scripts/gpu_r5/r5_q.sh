#!/bin/bash
# Round-5 GPU pass Q (rerun with overwrite-style gradients under ZeRO-1 too): ZeRO-1 trainer at world 2 / 4 on one GPU (peer-memory collectives, RCCL stream
# semantics) against world 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_multirank_gpu.py tests/test_determinism_gpu.py tests/test_train_gpu.py > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
echo done
