#!/bin/bash
# Round-5 GPU pass H: lora_xtg three-stage narrow path (default) vs two stages
# (MXLLM_LORA_XTG_STAGES=2): parity, per-projection probe, headline A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5h
mkdir -p $O
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "lora" tests/test_model_gpu.py -k "lora" > $O/lora_tests.log 2>&1 || { echo "lora tests failed"; tail -5 $O/lora_tests.log; exit 1; }
tail -1 $O/lora_tests.log
for i in 1 2; do
  for ST in 2 3; do
    MXLLM_LORA_XTG_STAGES=$ST timeout -k 10 200 python -u bench/lora_probe.py --tokens 4096 --wgs 256 --rounds 3 > $O/probe_st${ST}_$i.txt 2>&1 || { echo "probe failed"; exit 1; }
  done
done
grep -h "grads" $O/probe_st*_1.txt | head -20
for i in 1 2; do
  for ST in 2 3; do
    MXLLM_LORA_XTG_STAGES=$ST timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --config2 off --no-calibrate --json-out $O/head_st${ST}_$i.json > $O/head_st${ST}_$i.log 2>&1 || { echo "bench failed"; exit 1; }
    echo "stages $ST run $i: $(python -c "import json;j=json.load(open('$O/head_st${ST}_$i.json'));print(j['value'],j['ms_per_step'])")"
  done
done
echo done
