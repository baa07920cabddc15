#!/bin/bash
# Round-3 GPU pass O: the driver's round-end sequence on this tree (GPU suite, smoke(), default bench
# line) and a kernel-trace profile of the 70B LoRA headline step.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 600 python -u bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1
bash scripts/profile_bench.sh r3o/prof70b --steps 2 --warmup 1 --config2 off
python scripts/step_breakdown.py $O/prof70b/run_kernel_trace.csv 30 > $O/step_breakdown_70b.txt 2>&1 || true
timeout -k 10 300 python -u bench/dw_gemm_probe.py > $O/dw_probe_bf16.jsonl 2> $O/dw_probe.err || true
