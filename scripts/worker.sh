#!/usr/bin/env bash
# Worker-job entry for a cluster scheduler: LOCAL_RANK here is the NODE rank (reference contract),
# WORLD_SIZE the number of nodes, MASTER_IP=0 means "this host is the master".
set -euo pipefail
cd "$(dirname "$0")/.."
if [ "${MASTER_IP:-0}" == "0" ]; then MASTER_IP=127.0.0.1; fi
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec python ./modules/train.py --local_rank "$LOCAL_RANK" --dist_world_size "$WORLD_SIZE" --dist_backend nccl \
    --dist_init_method "tcp://${MASTER_IP}:${MASTER_PORT:-9080}" "$@"
