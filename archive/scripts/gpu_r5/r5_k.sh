#!/bin/bash
# Round-5 GPU pass K: config-4 proxy with the emulated collectives inline (default) vs on their own
# streams (MXLLM_Z3_EMUL_ASYNC=1, RCCL's stream semantics), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5k
mkdir -p $O
export PYTHONUNBUFFERED=1
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
for i in 1 2; do
  for A in 0 1; do
    MXLLM_Z3_EMUL_ASYNC=$A timeout -k 10 400 python -u bench.py $C4 --json-out $O/c4_async${A}_$i.json > $O/c4_async${A}_$i.log 2>&1 || { echo "c4 async=$A rc=$?"; tail -5 $O/c4_async${A}_$i.log; exit 1; }
    echo "async=$A run $i: $(python -c "import json;j=json.load(open('$O/c4_async${A}_$i.json'));print(j['ms_per_step'],j['value'],j['final_loss'],j['peak_hbm_reserved_gb'])")"
  done
done
echo done
