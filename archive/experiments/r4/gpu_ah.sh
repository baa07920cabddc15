#!/bin/bash
# round 4 pass AH: attention forward variants at the final tree (B2 / B16 S2048): DMA spreading flag,
# 8-wave workgroups, the pipelined kernel
OUT=gpurun_out/r4ah; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for V in "F=1 W=4" "F=0 W=4" "F=1 W=8" "P=p"; do
    set -- $V
    env_f=""; env_w=""; env_p=""
    case $V in *F=0*) env_f=0;; *F=1*) env_f=1;; esac
    case $V in *W=8*) env_w=8;; *W=4*) env_w=4;; esac
    case $V in *P=p*) env_p=p;; esac
    tag=$(echo $V | tr ' =' '__')
    MXLLM_ATTN_FWD_FLAGS=$env_f MXLLM_ATTN_FWD_WAVES=$env_w MXLLM_ATTN_FWD=$env_p timeout -k 10 120 python -u bench/attn_bench.py 2 64 8 2048 128 lite > $OUT/b2_${tag}_$i.txt 2>&1 || { echo "b2 $V rc=$?"; exit 1; }
    MXLLM_ATTN_FWD_FLAGS=$env_f MXLLM_ATTN_FWD_WAVES=$env_w MXLLM_ATTN_FWD=$env_p timeout -k 10 120 python -u bench/attn_bench.py 16 64 8 2048 128 lite > $OUT/b16_${tag}_$i.txt 2>&1 || { echo "b16 $V rc=$?"; exit 1; }
    echo "$V run $i: B2 fwd $(python -c "import json;j=json.loads(open('$OUT/b2_${tag}_$i.txt').read().strip().splitlines()[-1]);print(j['fwd_ms'])") B16 fwd $(python -c "import json;j=json.loads(open('$OUT/b16_${tag}_$i.txt').read().strip().splitlines()[-1]);print(j['fwd_ms'])")"
  done
done
