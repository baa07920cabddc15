set -e
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "lora_transposed" > gpurun_out/r2k_tests.log 2>&1
timeout -k 10 300 python bench/gemm_orient_probe.py > gpurun_out/r2k_orient.log 2>&1
timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2k_base.json 2>/dev/null
MXLLM_LORA_T=gu,d timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2k_t_gud.json 2>/dev/null
MXLLM_LORA_T=gu,d,qkv,o MXLLM_DX_IMAGE= timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2k_t_all.json 2>/dev/null
