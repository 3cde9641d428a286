#!/usr/bin/env bash
# Kernel-trace profile of the headline bench step (5 timed steps + 3 warmup).  Usage: tools/gpu/step_prof.sh <outdir> [bench args]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-step_prof}
shift || true
mkdir -p "$O"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 3 "$@" > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
cp "$S" "$O/run_kernel_stats.csv"
python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table.txt" 2>&1; head -30 "$O/kernel_table.txt"
