#!/usr/bin/env bash
# Steady-state kernel tables (bf16 and fp8) of the session-3 tree (tools/trace_steps.py: last 5 of 17 steps).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3b}
mkdir -p "$O"
for p in bf16 fp8; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$p" -o run -- python3 bench.py --steps 5 --warmup 12 --precision $p > "$O/prof_$p.log" 2>&1 || { tail -20 "$O/prof_$p.log"; exit 1; }
  T=$(find "$O/prof_$p" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_$p.txt" 2>&1
  head -16 "$O/steady_$p.txt"; tail -2 "$O/steady_$p.txt"
  rm -f "$T"
done
