#!/bin/bash
# Round-3 GPU pass H: the driver's round-end sequence on the current tree -- the whole GPU
# suite, smoke(), then the default bench line (headline + config 2).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 600 python -u bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1
