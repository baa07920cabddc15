#!/bin/bash
# Round-5 GPU pass S: clock / power / clock-normalised rate of gemm8 vs hipBLASLt under sustained load,
# and GRBM_GUI_ACTIVE cycles per dispatch (effective clock per kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5s
mkdir -p $O
export PYTHONUNBUFFERED=1
for S in o gu; do
  timeout -k 10 200 python -u bench/gemm_power_probe.py --shape $S --seconds 3 --rounds 2 > $O/power_$S.txt 2>$O/power_$S.err || { echo "probe rc=$?"; tail -5 $O/power_$S.err; exit 1; }
  cat $O/power_$S.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/pmc -o run -- python3 $R/bench/gemm_power_probe.py --shape o --seconds 0.3 --rounds 1 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
echo done
