#!/usr/bin/env bash
# torchrun env contract (RANK/LOCAL_RANK/WORLD_SIZE): NPROC workers on this node.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "${NPROC:-8}" --master-addr 127.0.0.1 \
    --master-port "${MASTER_PORT:-29500}" -m ml_recipe_distributed_pytorch_amd.cli.train "$@"
