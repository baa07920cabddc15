#!/bin/bash
# A/B of which LoRA projections keep a transposed [W; A] dX image (MXLLM_DX_IMAGE), 70B LoRA step.
set -e
timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_qkv_o.json 2>/dev/null
MXLLM_DX_IMAGE=qkv,d timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_qkv_d.json 2>/dev/null
MXLLM_DX_IMAGE=qkv,o,d timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_qkv_o_d.json 2>gpurun_out/r2n_qkv_o_d.err || true
MXLLM_DX_IMAGE=qkv,o,d timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r2n_qkv_o_d2.json 2>gpurun_out/r2n_qkv_o_d2.err || true
