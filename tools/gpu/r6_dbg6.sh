#!/usr/bin/env bash
# Graph divergence under the per-op sync proxy: with the HIP caching allocator disabled, and with the allocator's
# expandable segments off / garbage collection on, to test the allocator-aliasing hypothesis.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg6
mkdir -p "$O"
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1_$2.log" 2>&1; echo "$* rc=$? $(tail -1 "$O/$1_$2.log" | cut -c1-420)"; }
run HQ_SYNC_PROXY=1 PYTORCH_NO_HIP_MEMORY_CACHING=1 PYTORCH_NO_CUDA_MEMORY_CACHING=1
run HQ_SYNC_PROXY=1 X=again
