#!/bin/bash
# Round-5 GPU pass E: strict parity (half-ulp output allowance), config-4 proxy A/B of the
# persistent gemm8 on the fp32 dW shapes (table ph 5 vs MXLLM_GEMM8_PERSIST=0), whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5e
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_strict_parity_gpu.py > $O/strict.log 2>&1 || echo "strict parity: failures (see log)"
C4="--model llama3.1-70b --finetune full --parallel zero3 --act-ckpt --act-ckpt-layers 0 --micro-batch 4 --emulate-world 8 --steps 3 --warmup 2 --no-calibrate"
for i in 1 2; do
  for P in 0 table; do
    MXLLM_GEMM8_PERSIST=${P/table/} timeout -k 10 400 python -u bench.py $C4 --json-out $O/c4_p${P}_$i.json > $O/c4_p${P}_$i.log 2>&1 || { echo "c4 p=$P rc=$?"; exit 1; }
    echo "c4 persist=$P run $i: $(python -c "import json;j=json.load(open('$O/c4_p${P}_$i.json'));print(j['ms_per_step'],j['value'])")"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || { echo "gpu suite rc=$rc"; exit 1; }
echo done
