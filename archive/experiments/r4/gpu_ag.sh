#!/bin/bash
# round 4 pass AG: with the counted wait, are the wave priorities (bit 1) still worth it? 273 vs 272
OUT=gpurun_out/r4ag; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for P in 273 272; do
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/b2_${P}_$i.txt 2>&1 || { echo "b2 $P rc=$?"; exit 1; }
    MXLLM_ATTN_BWD8_PRIO=$P timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $OUT/b16_${P}_$i.txt 2>&1 || { echo "b16 $P rc=$?"; exit 1; }
    echo "prio $P run $i: B2 $(python -c "import json;j=json.loads(open('$OUT/b2_${P}_$i.txt').read().strip().splitlines()[-1]);print(j['bwd_ms'])") B16 $(python -c "import json;j=json.loads(open('$OUT/b16_${P}_$i.txt').read().strip().splitlines()[-1]);print(j['bwd_ms'])")"
  done
done
MXLLM_ATTN_BWD8_PRIO=272 MXLLM_ATTN_PROF=1 timeout -k 10 200 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/prof_272.txt 2>&1 || { echo "prof rc=$?"; exit 1; }
grep -v "^{" $OUT/prof_272.txt | tail -3
