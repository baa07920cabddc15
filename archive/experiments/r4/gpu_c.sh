#!/bin/bash
# round 4 pass C: gemm8 win table (probe incl. the 70B LoRA augmented shapes, T 4096; fp32 dW at T 8192),
# then a same-box A/B of the bench line with / without the table, then PMC counters of gemm8's forms
OUT=gpurun_out/r4c; mkdir -p $OUT
ROOT=$(pwd)
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench/gemm8_probe.py --aug --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_t4096.json > $OUT/probe_t4096.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
timeout -k 10 300 python -u bench/gemm8_probe.py --model 70b --tokens 8192 --forms tt32 --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_t8192.json > $OUT/probe_t8192.txt 2>&1 || { echo "probe8k rc=$?"; exit 1; }
tail -2 $OUT/probe_t8192.txt
cp $OUT/gemm8_gfx950.json mxllm/tuning/gemm8_gfx950.json
for i in 1 2; do
  MXLLM_GEMM8=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/bench_off_$i.json 2> $OUT/bench_off_$i.err || { echo "bench off rc=$?"; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config2-mb4 off > $OUT/bench_on_$i.json 2> $OUT/bench_on_$i.err || { echo "bench on rc=$?"; exit 1; }
  echo "off $i: $(python -c "import json;j=json.load(open('$OUT/bench_off_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")  on $i: $(python -c "import json;j=json.load(open('$OUT/bench_on_$i.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/$OUT/p1 -o p1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -- python3 $ROOT/bench/gemm8_probe.py --model 70b --shapes o --forms nn,tt,tn --rounds 1 --calls 2 --no-table > $ROOT/$OUT/p1.log 2>&1 || { echo "pmc1 rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/$OUT/p2 -o p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -- python3 $ROOT/bench/gemm8_probe.py --model 70b --shapes o --forms nn,tt,tn --rounds 1 --calls 2 --no-table > $ROOT/$OUT/p2.log 2>&1 || { echo "pmc2 rc=$?"; exit 1; }
python3 $ROOT/scripts/pmc_summary.py $ROOT/$OUT gemm8 Cijk > $ROOT/$OUT/pmc_summary.txt 2>&1; tail -30 $ROOT/$OUT/pmc_summary.txt
