#!/bin/bash
# round 5 last check at the final tree (AdamW grid cap 1,024): train / kernel suites, smoke, default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5_final6
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_determinism_gpu.py tests/test_kernels_gpu.py -k "adamw or train or determin or overlapped" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$O/bench.json'));print(j['value'],j['ms_per_step'],j['config2_8b_full']['value'],j['config2_8b_full']['ms_per_step'],j['config2_8b_full_mb4']['value'],j['calibration'])"
echo done
