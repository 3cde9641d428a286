#!/usr/bin/env bash
# Steady-state kernel tables (last 5 steps after 12 warm-up / calibration steps): fp8 and bf16.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_f
mkdir -p "$O"
for p in fp8 bf16; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$p" -o run -- python3 bench.py --precision $p --steps 5 --warmup 12 > "$O/prof_$p.log" 2>&1 || { tail -20 "$O/prof_$p.log"; exit 1; }
  T=$(find "$O/prof_$p" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_$p.txt" 2>&1
  head -40 "$O/steady_$p.txt"; tail -2 "$O/steady_$p.txt"
  rm -f "$T"
done
