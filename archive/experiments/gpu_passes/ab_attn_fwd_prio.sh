#!/bin/bash
set -e
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2t_tests.log 2>&1
MXLLM_ATTN_FWD_WAVES=8 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2t_tests8.log 2>&1
timeout -k 10 120 python bench/attn_bench.py > gpurun_out/r2t_attn4.json 2>/dev/null
MXLLM_ATTN_FWD_WAVES=8 timeout -k 10 120 python bench/attn_bench.py > gpurun_out/r2t_attn8prio.json 2>/dev/null
