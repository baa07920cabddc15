#!/bin/bash
# Round-3 GPU pass C: new GPU tests (paged KV, sampler workspace, split master), the 8B
# serving bench static vs paged KV, the 8B ZeRO-3 vs DDP world-1 gap and the config-4
# world-8 emulated proxy (fp32 reduce-scatter, split master).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
timeout -k 10 300 python bench/serve_bench.py --model llama3.1-8b --batches 1,8,64 --requests 64 --json-out $O/serve8b_static.json > $O/serve8b_static.log 2>&1
timeout -k 10 300 python bench/serve_bench.py --model llama3.1-8b --batches 1,8,64 --requests 64 --kv-pool-tokens 98304 --json-out $O/serve8b_paged.json > $O/serve8b_paged.log 2>&1
timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --parallel zero3 --steps 10 --warmup 3 --json-out $O/8b_zero3.json > $O/8b_zero3.log 2>&1
timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --steps 10 --warmup 3 --json-out $O/8b_ddp.json > $O/8b_ddp.log 2>&1
timeout -k 10 400 python bench.py --model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 56 --micro-batch 4 --emulate-world 8 --steps 2 --warmup 1 --json-out $O/z3emu8.json > $O/z3emu8.log 2>&1
