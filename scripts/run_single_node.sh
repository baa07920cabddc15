#!/bin/bash
# One node, one process per GPU (or NPROC_PER_NODE CPU processes on gloo).
# usage: scripts/run_single_node.sh [program args...]   (SCRIPT=src/distributed_inference.py to serve)
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
if [ -z "${NPROC_PER_NODE:-}" ]; then
  NPROC_PER_NODE=$(python3 -c "import torch;print(max(1,torch.cuda.device_count()))" 2>/dev/null || echo 1)
fi
exec python3 -m torch.distributed.run --standalone --nnodes=1 --nproc_per_node=${NPROC_PER_NODE} \
  --master_addr=127.0.0.1 --max-restarts=${MAX_RESTARTS:-0} ${SCRIPT:-src/distributed_finetuning.py} "$@"
