#!/bin/bash
# round 4 pass G: (1) gemm8 win table at T 8192 (config 4 / config-2 mb4 / 8B S 8k shapes, incl. the
# 70B LM head); (2) config-4 proxy at 56 / 40 / 24 checkpointed layers with the new table;
# (3) kernel-trace step breakdowns of the headline and the config-4 proxy (no Cijk_Ailk / transpose16?)
OUT=gpurun_out/r4g; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cp mxllm/tuning/gemm8_gfx950.json $OUT/gemm8_gfx950.json
timeout -k 10 500 python -u bench/gemm8_probe.py --model both --tokens 8192 --forms nn,tt,tt32,tn --ph4 --rounds 3 --write-table $OUT/gemm8_gfx950.json --json-out $OUT/probe_t8192.json > $OUT/probe_t8192.txt 2>&1 || { echo "probe8k rc=$?"; exit 1; }
tail -1 $OUT/probe_t8192.txt
cp $OUT/gemm8_gfx950.json mxllm/tuning/gemm8_gfx950.json
for CK in 56 40 24; do
  C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers $CK --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
  timeout -k 10 400 python -u bench.py $C4 --json-out $OUT/c4_ck$CK.json > $OUT/c4_ck$CK.log 2>&1 || { echo "c4 ck$CK rc=$?"; exit 1; }
  echo "c4 ck$CK: $(python -c "import json;j=json.load(open('$OUT/c4_ck$CK.json'));print(j['ms_per_step'],j['value'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])")"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; exit 1; }
echo "bench: $(python -c "import json;j=json.load(open('$OUT/bench.json'));print(j['ms_per_step'],j['config2_8b_full']['ms_per_step'],j['config2_8b_full_mb4']['ms_per_step'],j['calibration'])")"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_head -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --config2 off --no-calibrate > $ROOT/$OUT/prof_head.log 2>&1 || { echo "prof head rc=$?"; exit 1; }
python $ROOT/scripts/step_breakdown.py $ROOT/$OUT/prof_head/run_kernel_trace.csv 30 > $ROOT/$OUT/step_breakdown_70b_lora.txt
head -12 $ROOT/$OUT/step_breakdown_70b_lora.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_8b -o run -- python3 $ROOT/bench.py --model llama3.1-8b --finetune full --steps 3 --warmup 1 --no-calibrate > $ROOT/$OUT/prof_8b.log 2>&1 || { echo "prof 8b rc=$?"; exit 1; }
python $ROOT/scripts/step_breakdown.py $ROOT/$OUT/prof_8b/run_kernel_trace.csv 30 > $ROOT/$OUT/step_breakdown_8b_full.txt
head -12 $ROOT/$OUT/step_breakdown_8b_full.txt
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_c4 -o run -- python3 $ROOT/bench.py --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 2 --warmup 1 --no-calibrate > $ROOT/$OUT/prof_c4.log 2>&1 || { echo "prof c4 rc=$?"; exit 1; }
python $ROOT/scripts/step_breakdown.py $ROOT/$OUT/prof_c4/run_kernel_trace.csv 30 > $ROOT/$OUT/step_breakdown_c4.txt
head -12 $ROOT/$OUT/step_breakdown_c4.txt
rm -f $ROOT/$OUT/prof_*/run_kernel_trace.csv.gz
du -sh $ROOT/$OUT
