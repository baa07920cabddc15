#!/bin/bash
# round 5: the whole GPU suite once more at the final tree (AdamW grid cap 1,024)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5_final7
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || { echo "gpu suite rc=$rc"; grep -E "FAILED|^E " $O/tests.txt | head -20; exit 1; }
echo done
