#!/usr/bin/env bash
# Build and run the attention lab on the GPU box: bash tools/attn_lab/run.sh [B]
set -eo pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/attn_lab
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iml_recipe_distributed_pytorch_amd/csrc/include \
  tools/attn_lab/attn_lab.hip -o gpurun_out/attn_lab/attn_lab
timeout -k 10 120 gpurun_out/attn_lab/attn_lab "${1:-256}" | tee gpurun_out/attn_lab/out.txt
