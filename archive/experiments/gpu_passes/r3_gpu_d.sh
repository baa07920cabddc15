#!/bin/bash
# Round-3 GPU pass D: ZeRO-3 without AdamW gradient zeroing (first write of a step
# overwrites the fp32 grad shard): 8B ZeRO-3 vs DDP at world 1 in both gradient dtypes,
# the config-4 emulated proxy and its kernel profile (no fold / transpose accounting).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_kvcache.py tests/test_model_gpu.py > $O/tests.log 2>&1
B="python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3"
for gd in fp32 bf16; do
  timeout -k 10 200 $B --parallel zero3 --grad-dtype $gd --json-out $O/8b_zero3_$gd.json > $O/8b_zero3_$gd.log 2>&1
  timeout -k 10 200 $B --parallel ddp --grad-dtype $gd --json-out $O/8b_ddp_$gd.json > $O/8b_ddp_$gd.log 2>&1
done
timeout -k 10 400 python bench.py --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 2 --warmup 1 --json-out $O/z3emu8.json > $O/z3emu8.log 2>&1
bash scripts/profile_bench.sh r3d/prof_z3emu --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 2 --warmup 1
python scripts/step_breakdown.py $O/prof_z3emu/run_kernel_trace.csv 30 > $O/z3emu_breakdown.txt 2>&1 || true
for v in 1 0; do
  MXLLM_MERGE_FUSED=$v timeout -k 10 300 python bench/serve_bench.py --model llama3.1-8b --batches 1,4,64 --requests 0 --json-out $O/serve8b_merge$v.json > $O/serve8b_merge$v.log 2>&1
done
