#!/bin/bash
# round 4 long context, final tree: 8B full fine-tune at S = 32k with no checkpointed layer and the
# activation recompute (--act-ckpt --act-ckpt-layers 0), S = 64k with every layer checkpointed, and the
# attention kernels at 8k / 32k (the backward with the counted end-of-tile wait)
OUT=gpurun_out/r4_long2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for S in 8192 32768; do
  timeout -k 10 200 python -u bench/attn_bench.py 1 32 8 $S 128 lite > $OUT/attn_8b_S$S.txt 2>&1 || { echo "attn $S rc=$?"; exit 1; }
  echo "attn 8B heads S=$S: $(grep shape $OUT/attn_8b_S$S.txt)"
done
S=32768
timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt --act-ckpt-layers 0 \
   --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_recompute.json > $OUT/8b_full_S${S}_recompute.log 2>&1
rc=$?; echo "S=$S recompute rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_recompute.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 \
   --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_nockpt.json > $OUT/8b_full_S${S}_nockpt.log 2>&1
rc=$?; echo "S=$S no ckpt rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_nockpt.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
[ $rc -eq 0 ] || exit $rc
S=65536
timeout -k 10 600 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt \
   --steps 2 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_ckpt.json > $OUT/8b_full_S${S}_ckpt.log 2>&1
rc=$?; echo "S=$S every layer ckpt rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_ckpt.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
exit $rc
