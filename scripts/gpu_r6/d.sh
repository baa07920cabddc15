#!/bin/bash
# r6 pass D: config-4 proxy with the recompute path through the fused gate-up + SwiGLU epilogues
# (MXLLM_REC_FUSED=1, new default) vs the unfused recompute (0), alternating; then a kernel trace of =1.
set -o pipefail
OUT=gpurun_out/r6d; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_epi_gpu.py > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
for run in 1 0 1 0; do
  tag=rf${run}_$((++i))
  MXLLM_REC_FUSED=$run timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/c4_$tag.json > $OUT/c4_$tag.log 2>&1 || { echo "c4 $tag rc=$?"; tail -5 $OUT/c4_$tag.log; exit 1; }
  echo "c4 $tag: $(python -c "import json;j=json.load(open('$OUT/c4_$tag.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_reserved_gb'])")"
done
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $ROOT/$OUT/prof_c4 -o run -- python3 $ROOT/bench.py $C4 > $ROOT/$OUT/prof_c4.log 2>&1 || { echo "prof c4 rc=$?"; exit 1; }
cd $ROOT
python scripts/step_breakdown.py $OUT/prof_c4/run_kernel_trace.csv 40 embedding_fwd > $OUT/step_breakdown_c4_ck0.txt
head -24 $OUT/step_breakdown_c4_ck0.txt
rm -f $OUT/prof_c4/run_kernel_trace.csv
