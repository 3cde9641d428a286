#!/usr/bin/env bash
# Release kernels behind the per-op sync proxy (HQ_SYNC_PROXY=1): does the graph-run divergence follow the
# proxy's synchronisation or the debug kernels?  Plus the two-op sync subsets of the optimizer phase.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg5
mkdir -p "$O"
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1_$2.log" 2>&1; echo "$* rc=$? $(tail -1 "$O/$1_$2.log" | cut -c150-400)"; }
run HQ_SYNC_PROXY=1 X=all
run HQ_SYNC_PROXY=1 HQ_DEBUG_SYNC_ONLY=sq_norm_chunks,clip_from_partials,adamw
run HQ_KERNELS_DEBUG=1 HQ_DEBUG_SYNC_ONLY=sq_norm_chunks,clip_from_partials,adamw
run HQ_KERNELS_DEBUG=1 HQ_DEBUG_SYNC_ONLY=clip_from_partials,adamw
