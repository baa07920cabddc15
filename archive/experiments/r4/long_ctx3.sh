#!/bin/bash
# round 4: 8B full fine-tune at S = 64k, selective checkpointing with the activation recompute in the
# un-checkpointed layers (16 / 8 of 32 checkpointed)
OUT=gpurun_out/r4_long2; mkdir -p $OUT
export PYTHONUNBUFFERED=1
S=65536
for CK in 16 8; do
  timeout -k 10 600 python -u bench.py --model llama3.1-8b --finetune full --seq-len $S --micro-batch 1 --act-ckpt --act-ckpt-layers $CK \
     --steps 2 --warmup 1 --config2 off --no-calibrate --json-out $OUT/8b_full_S${S}_ck$CK.json > $OUT/8b_full_S${S}_ck$CK.log 2>&1
  rc=$?; echo "S=$S ck$CK rc=$rc: $(python -c "import json;j=json.load(open('$OUT/8b_full_S${S}_ck$CK.json'));print(j['ms_per_step'],j['value'],j['mfu_vs_2.5PF_dense'],j['peak_hbm_gb'],j['peak_hbm_reserved_gb'])" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 $OUT/8b_full_S${S}_ck$CK.log; exit $rc; }
done
