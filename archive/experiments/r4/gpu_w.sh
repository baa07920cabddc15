#!/bin/bash
# round 4 pass W: fp8-weight decode (e4m3 projections, csrc/kernels/fp8_gemm.hip) at the current
# tree -- 70B / 8B engine numbers and a kernel profile of the 70B fp8 decode
OUT=gpurun_out/r4w; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench/serve_bench.py --model llama3.1-70b --fp8 --batches 1,8,64 --requests 16 --json-out $OUT/serve70b_fp8.json > $OUT/serve70b_fp8.log 2>&1 || { echo "serve 70b fp8 rc=$?"; tail -5 $OUT/serve70b_fp8.log; exit 1; }
python -c "import json;j=json.load(open('$OUT/serve70b_fp8.json'));print('70b fp8', j['prefill'], [(d['batch'], d['ms_per_step']) for d in j['decode']])"
timeout -k 10 300 python -u bench/serve_bench.py --model llama3.1-8b --fp8 --batches 1,8,64 --requests 16 --json-out $OUT/serve8b_fp8.json > $OUT/serve8b_fp8.log 2>&1 || { echo "serve 8b fp8 rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$OUT/serve8b_fp8.json'));print('8b fp8', j['prefill'], [(d['batch'], d['ms_per_step']) for d in j['decode']])"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof70 -o run -- python3 $ROOT/bench/serve_bench.py --model llama3.1-70b --fp8 --batches 1 --requests 4 --decode-steps 16 > $ROOT/$OUT/prof70.log 2>&1 || { echo "prof rc=$?"; exit 1; }
head -12 $ROOT/$OUT/prof70/run_kernel_stats.csv | cut -c1-150
rm -f $ROOT/$OUT/prof70/run_kernel_trace.csv
