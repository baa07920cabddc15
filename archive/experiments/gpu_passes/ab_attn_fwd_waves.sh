set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or engine or prefill or ring" > gpurun_out/r2l_tests.log 2>&1
timeout -k 10 120 python bench/attn_bench.py > gpurun_out/r2l_attn4.json 2>/dev/null
MXLLM_ATTN_FWD_WAVES=8 timeout -k 10 120 python bench/attn_bench.py > gpurun_out/r2l_attn8.json 2>/dev/null
