#!/usr/bin/env bash
# Synced graph divergence: does a device sync between the replay's input copies / seed fill and the graph launch
# remove it?
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg8
mkdir -p "$O"
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1_$2.log" 2>&1; echo "$* rc=$? $(tail -1 "$O/$1_$2.log" | cut -c150-420)"; }
run HQ_SYNC_PROXY=1 HQ_LAB_SYNC_BEFORE_REPLAY=1
run HQ_LAB_SYNC_BEFORE_REPLAY=1 X=1
