#!/bin/bash
# r6 pass N: kernel trace of the headline step at the last round-6 tree (70B LoRA, 1 GPU) -> per-kernel and per-call breakdowns.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r6n
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 $ROOT/bench.py --steps 2 --warmup 1 --config2 off --no-calibrate > $OUT/bench.log 2>&1 \
  || { tail -20 $OUT/bench.log; exit 1; }
cd $ROOT
CSV=$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1)
python scripts/step_breakdown.py $CSV 40 > $OUT/step_breakdown.txt
for k in lora_xtg lora_xwt swiglu_lora Cijk gemm8_kernel g8_sum2 attn_fwd attn_bwd8 attn_bwd_dq rmsnorm rope; do
  python scripts/kernel_calls.py $CSV $k >> $OUT/calls.txt
done
head -25 $OUT/step_breakdown.txt
cat $OUT/calls.txt
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
rm -f $CSV
