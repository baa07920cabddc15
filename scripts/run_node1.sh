#!/bin/bash
# Node 1 of a multi-node mxllm job (reference scripts/run_node1.sh, MI355X/RCCL edition).
#
# Same torchrun contract as the reference (nproc_per_node, nnodes, node_rank,
# master_addr, master_port), every value overridable by env:
#   NPROC_PER_NODE (default: all local GPUs, or 1 on CPU)  NNODES (2)
#   MASTER_ADDR (127.0.0.1)  MASTER_PORT (29500)  SCRIPT (src/distributed_finetuning.py)
#   MAX_RESTARTS (0)  RDZV_BACKEND (static; set c10d for elastic restarts)
# Single-box 2-node emulation (BASELINE config 5): run both scripts on one
# 8xMI355X host with HIP_VISIBLE_DEVICES=0,1,2,3 / 4,5,6,7 and NPROC_PER_NODE=4.
# Extra arguments are passed to the training/inference program.
set -euo pipefail
cd "$(dirname "$0")/.."

# RCCL transport: inside a node RCCL uses xGMI peer links; between nodes it uses
# RoCE/IB when present, else sockets on NCCL_SOCKET_IFNAME (RCCL honours NCCL_*).
export NCCL_SOCKET_IFNAME=${NCCL_SOCKET_IFNAME:-$(ip -o -4 route show to default 2>/dev/null | awk '{print $5}' | head -n1)}
export NCCL_IB_DISABLE=${NCCL_IB_DISABLE:-1}
export NCCL_DEBUG=${NCCL_DEBUG:-WARN}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
# Completion endpoint for the inference driver: "local" = this rank's own GPU.
export MXLLM_API_BASE=${MXLLM_API_BASE:-local}
# export OPENAI_API_KEY=...   # only needed for a remote OpenAI-compatible endpoint

if [ -z "${NPROC_PER_NODE:-}" ]; then
  NPROC_PER_NODE=$(python3 -c "import torch;print(max(1,torch.cuda.device_count()))" 2>/dev/null || echo 1)
fi

exec python3 -m torch.distributed.run \
  --nproc_per_node=${NPROC_PER_NODE} \
  --nnodes=${NNODES:-2} \
  --node_rank=1 \
  --master_addr=${MASTER_ADDR:-127.0.0.1} \
  --master_port=${MASTER_PORT:-29500} \
  --max-restarts=${MAX_RESTARTS:-0} \
  --rdzv-backend=${RDZV_BACKEND:-static} \
  ${SCRIPT:-src/distributed_finetuning.py} "$@"
