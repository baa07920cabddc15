#!/bin/bash
# round 5 long context at the final tree: 8B full fine-tune, one sequence per step, S = 32k without
# checkpointing and with the activation recompute, S = 64k with the first 16 layers checkpointed
OUT=gpurun_out/r5_long; mkdir -p $OUT
export PYTHONUNBUFFERED=1
S=32768
for V in nockpt recompute; do
  X=""; [ $V = recompute ] && X="--act-ckpt --act-ckpt-layers 0"
  timeout -k 10 400 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 $X \
     --steps 3 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_$V.json > $OUT/8b_full_S${S}_$V.log 2>&1
  rc=$?; echo "S=$S $V rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_$V.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
S=65536
timeout -k 10 600 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt --act-ckpt-layers 16 \
   --steps 2 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_ck16.json > $OUT/8b_full_S${S}_ck16.log 2>&1
rc=$?; echo "S=$S ck16 rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_ck16.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
[ $rc -eq 0 ] || exit $rc
echo done
