#!/bin/bash
# A/B of the newest tuned-table entry (last line) on the 70B LoRA headline, same box.
set -e
O=gpurun_out/abtab; mkdir -p $O
head -n -1 mxllm/tuning/tunableop_gfx950.csv > /tmp/prev_table.csv
for v in new prev new prev; do
  if [ $v = prev ]; then export MXLLM_GEMM_TABLE=/tmp/prev_table.csv; else unset MXLLM_GEMM_TABLE; fi
  timeout -k 10 400 python bench.py --steps 6 --warmup 2 --json-out $O/$v.json > $O/$v.log 2>&1
  python -c "import json;d=json.load(open('$O/$v.json'));print('$v',d['value'],d['ms_per_step'])" >> $O/summary.txt
done
