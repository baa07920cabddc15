#!/bin/bash
# Headline scaling curve: bench.py at 1, 2, 4, 8 GPUs back to back (one node).
# usage: scripts/bench_scaling.sh [bench args...]  -> gpurun_out/scale_<N>.json
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
NG=$(python3 -c "import torch;print(torch.cuda.device_count())")
PORT=${MASTER_PORT:-29700}
for N in 1 2 4 8; do
  [ "$N" -le "$NG" ] || break
  if [ "$N" -eq 1 ]; then
    timeout -k 10 1200 python3 bench.py --gpus 1 --json-out gpurun_out/scale_1.json "$@"
  else
    timeout -k 10 1200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((PORT + N)) bench.py --gpus $N --json-out gpurun_out/scale_$N.json "$@"
  fi
done
