#!/usr/bin/env bash
# One node, one worker process per visible MI355X (RCCL over xGMI).  Extra args go to train.py,
# e.g.  scripts/run_distributed_on_single_node.sh -c config/test_bert.cfg
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec python ./modules/train.py --local_rank 0 --dist_backend nccl \
    --dist_init_method "tcp://127.0.0.1:${MASTER_PORT:-9080}" "$@"
