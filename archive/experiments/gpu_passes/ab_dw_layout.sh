set -e
O=gpurun_out/abdw; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -q -x -k "train_step or bench_contract" > $O/tests.log 2>&1
for tn in 0 1; do
  MXLLM_DW_TN=$tn timeout -k 10 300 python bench.py --model llama3.1-8b --finetune full --steps 5 --warmup 2 --json-out $O/8b_tn$tn.json > $O/8b_tn$tn.log 2>&1
  MXLLM_DW_TN=$tn timeout -k 10 300 python bench.py --model llama3.1-70b --finetune full --parallel zero3 --layers 10 --steps 3 --warmup 1 --json-out $O/z3_tn$tn.json > $O/z3_tn$tn.log 2>&1
done
