#!/usr/bin/env bash
# Run on EVERY node (same GPU count per node).  NODE_RANK = this node's index, NNODES = node count,
# MASTER_IP/MASTER_PORT = node 0's address.  Each node spawns one worker per local GPU.
set -euo pipefail
cd "$(dirname "$0")/.."
: "${NODE_RANK:?set NODE_RANK}" "${NNODES:?set NNODES}" "${MASTER_IP:?set MASTER_IP}"
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec python ./modules/train.py --local_rank "$NODE_RANK" --dist_world_size "$NNODES" --dist_backend nccl \
    --dist_init_method "tcp://${MASTER_IP}:${MASTER_PORT:-9080}" "$@"
