#!/bin/bash
# round 6 serving evidence at the final tree: 8B / 70B engine numbers (paged KV default), 8B fp8,
# the reference's own inference program on the local 8B engine, and one long prompt (8k tokens:
# the reviews are no longer truncated)
OUT=gpurun_out/r6_serve; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench/serve_bench.py --model llama3.1-8b --json-out $OUT/serve8b.json > $OUT/serve8b.log 2>&1 || { echo "serve 8b rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$OUT/serve8b.json'));print('8b', j['prefill'], [(d['batch'], d['ms_per_step']) for d in j['decode']], j['e2e']['output_tokens_per_s'])"
timeout -k 10 300 python -u bench/serve_bench.py --model llama3.1-8b --prompt-len 8192 --batches 1 --ctx 8192 --requests 8 --json-out $OUT/serve8b_8k.json > $OUT/serve8b_8k.log 2>&1 || { echo "serve 8b 8k rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$OUT/serve8b_8k.json'));print('8b 8k', j['prefill'], [(d['batch'], d['ms_per_step']) for d in j['decode']])"
timeout -k 10 400 python -u bench/serve_bench.py --model llama3.1-70b --batches 1,64 --json-out $OUT/serve70b.json > $OUT/serve70b.log 2>&1 || { echo "serve 70b rc=$?"; exit 1; }
python -c "import json;j=json.load(open('$OUT/serve70b.json'));print('70b', j['prefill'], [(d['batch'], d['ms_per_step']) for d in j['decode']], j['e2e']['output_tokens_per_s'])"
MXLLM_ENGINE_MODEL=llama3.1-8b timeout -k 10 400 python -u bench/inference_workload.py > $OUT/reference_workload_8b.json 2> $OUT/reference_workload_8b.err || { echo "workload rc=$?"; tail -5 $OUT/reference_workload_8b.err; exit 1; }
tail -1 $OUT/reference_workload_8b.json
echo done
