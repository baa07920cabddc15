#!/bin/bash
# Round-5 GPU pass D: strict parity with the flash-formulation dQ/dK reference, fused-epilogue GEMMs
# in isolation, persistent gemm8 on the config-4 fp32-output dW shapes (T = 8192).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5d
mkdir -p $O
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_strict_parity_gpu.py > $O/strict.log 2>&1 || echo "strict parity: failures (see log)"
timeout -k 10 300 python -u bench/fused_epi_bench.py --tokens 4096 --rounds 5 > $O/fused_epi_t4096.txt 2>&1 || { echo "fused epi bench failed"; exit 1; }
timeout -k 10 420 python -u bench/gemm8_probe.py --model 70b --tokens 8192 --rounds 3 --forms tt32 --ph4 --persist --write-table $O/tt32_t8192_table.json > $O/probe70_tt32_t8192.txt 2>&1 || { echo "probe failed"; exit 1; }
echo done
