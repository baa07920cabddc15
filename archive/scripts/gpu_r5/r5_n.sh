#!/bin/bash
# Round-5 GPU pass N: dQ kernel with 128 q rows per workgroup and a 4-deep ring (MXLLM_ATTN_DQ_QB=2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5n
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
MXLLM_ATTN_DQ_QB=2 timeout -k 10 400 $T tests/test_attn_dqkv_gpu.py tests/test_strict_parity_gpu.py tests/test_kernels_gpu.py -k "attn or attention" > $O/tests_qb2.log 2>&1
rc=$?; tail -2 $O/tests_qb2.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; grep -E "FAILED|^E " $O/tests_qb2.log | head -20; exit 1; }
for i in 1 2; do
  for Q in 4 2; do
    MXLLM_ATTN_DQ_QB=$Q timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/attn_qb${Q}_$i.json 2>$O/attn_qb${Q}_$i.err || { echo "attn rc=$?"; exit 1; }
    echo "qb=$Q run $i: $(cat $O/attn_qb${Q}_$i.json)"
  done
done
cd /tmp && export TMPDIR=/tmp
for Q in 4 2; do
  MXLLM_ATTN_DQ_QB=$Q timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qb$Q -o run -- python3 $R/bench/attn_bench.py 2 64 8 2048 128 lite > $O/prof_qb$Q.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  grep -E "attn_bwd_dq|attn_bwd8|Name" $O/prof_qb$Q/run_kernel_stats.csv | cut -c1-200
  rm -f $O/prof_qb$Q/run_kernel_trace.csv
done
echo done
