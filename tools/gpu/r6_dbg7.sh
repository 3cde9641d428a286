#!/usr/bin/env bash
# Allocator-aliasing test for the synced graph divergence: keep every tensor any kernel op touched alive.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg7
mkdir -p "$O"
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1_$2.log" 2>&1; echo "$* rc=$? $(tail -1 "$O/$1_$2.log" | cut -c150-420)"; }
run HQ_SYNC_PROXY=1 HQ_PROXY_KEEP=1
run HQ_SYNC_PROXY=1 HQ_DEBUG_SYNC_ONLY=clip_from_partials,adamw HQ_PROXY_KEEP=1
