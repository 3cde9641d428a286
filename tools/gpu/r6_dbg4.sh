#!/usr/bin/env bash
# Bisect the debug-proxy graph mismatch: which ops' per-op synchronisation changes the graph run's result.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg4
mkdir -p "$O"
export HQ_KERNELS_DEBUG=1
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1.log" 2>&1; echo "$1 rc=$? $(tail -1 "$O/$1.log" | cut -c1-400)"; }
run HQ_DEBUG_SYNC_SKIP=sq_norm_chunks,clip_from_partials,adamw
run HQ_DEBUG_SYNC_ONLY=adamw
run HQ_DEBUG_SYNC_ONLY=sq_norm_chunks
run HQ_DEBUG_SYNC_ONLY=clip_from_partials
