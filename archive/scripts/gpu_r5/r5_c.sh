#!/bin/bash
# Round-5 GPU pass C: strict parity (all), staggered attention backward parity + timing, persistent
# gemm8 probes, config-2 kernel profile fused vs unfused epilogues.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5c
mkdir -p $O
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_strict_parity_gpu.py > $O/strict.log 2>&1 || echo "strict parity: failures (see log)"
MXLLM_ATTN_BWD8=2 timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" tests/test_strict_parity_gpu.py -k "attention" > $O/attn_bwd_stag.log 2>&1 || echo "bwd stagger parity: failures"
for i in 1 2; do
  for BW in 1 2; do
    MXLLM_ATTN_BWD8=$BW timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $O/bwd_b2_bw${BW}_$i.txt 2>&1 || { echo "bwd bench failed"; exit 1; }
    MXLLM_ATTN_BWD8=$BW timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $O/bwd_b16_bw${BW}_$i.txt 2>&1 || { echo "bwd bench16 failed"; exit 1; }
  done
done
timeout -k 10 420 python -u bench/gemm8_probe.py --model 70b --tokens 4096 --rounds 3 --forms tn,nn,tt32 --aug --ph4 --persist > $O/probe70_t4096.txt 2>&1 || { echo "probe 70b failed"; exit 1; }
timeout -k 10 300 python -u bench/gemm8_probe.py --model 8b --tokens 4096 --rounds 3 --forms tn,nn,tt --ph4 --persist > $O/probe8_t4096.txt 2>&1 || { echo "probe 8b failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  MXLLM_FUSED_EPI=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fused$f -o run -- python3 $R/bench.py --model llama3.1-8b --finetune full --steps 4 --warmup 2 --no-calibrate --config2 off --json-out $O/prof_fused$f.json > $O/prof_fused$f.log 2>&1 || { echo "rocprof fused=$f failed"; exit 1; }
done
echo done
