#!/bin/bash
# Round-3 GPU pass K: the reference's inference program (src/distributed_inference.py main(),
# 750 IMDB-like prompts) on the current 8B engine, and the 8B serving bench.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3k
mkdir -p $O
MXLLM_ENGINE_MODEL=llama3.1-8b timeout -k 10 400 python -u bench/inference_workload.py > $O/ref_workload_8b.log 2>&1
timeout -k 10 400 python -u bench/serve_bench.py --model llama3.1-8b --json-out $O/serve8b.json > $O/serve8b.log 2>&1
