#!/usr/bin/env bash
# Which side of the debug-build graph mismatch is off: losses of eager / graph runs for the release library,
# the debug library, and the debug library without its per-op synchronisation.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg3
mkdir -p "$O"
timeout -k 10 200 python tools/graph_losses.py > "$O/release.log" 2>&1; echo "release rc=$?"; tail -1 "$O/release.log"
HQ_KERNELS_DEBUG=1 timeout -k 10 200 python tools/graph_losses.py > "$O/debug.log" 2>&1; echo "debug rc=$?"; tail -1 "$O/debug.log"
HQ_KERNELS_DEBUG=1 HQ_DEBUG_NOSYNC=1 timeout -k 10 200 python tools/graph_losses.py > "$O/debug_nosync.log" 2>&1; echo "debug_nosync rc=$?"; tail -1 "$O/debug_nosync.log"
