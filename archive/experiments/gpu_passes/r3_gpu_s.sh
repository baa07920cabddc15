#!/bin/bash
# Round-3 GPU pass S: dW ring form with three stages in flight -- tests + probe
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k dw_gemm -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench/dw_gemm_probe.py > $O/probe_bf16.jsonl 2> $O/probe.err
