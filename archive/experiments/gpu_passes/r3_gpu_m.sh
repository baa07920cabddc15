#!/bin/bash
# Round-3 GPU pass M: token-major dW MFMA kernel (csrc/kernels/dw_gemm.hip) -- numerics tests,
# per-shape timing vs transpose + hipBLASLt TN / hipBLASLt NT, then the 8B full step A/B.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k dw_gemm -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench/dw_gemm_probe.py > $O/probe_bf16.jsonl 2> $O/probe_bf16.err
timeout -k 10 300 python -u bench/dw_gemm_probe.py --f32 --models 70b > $O/probe_f32.jsonl 2> $O/probe_f32.err
