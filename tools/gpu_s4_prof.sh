#!/usr/bin/env bash
# per-kernel table + idle-gap accounting of the default (b256) bench step after the session-4 kernels
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/s4_prof
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
S=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
T=$(find $O/prof -name 'run_kernel_trace.csv' | head -1)
python tools/kernel_table.py "$S" --steps 11 > $O/kernel_table.txt 2>&1; cat $O/kernel_table.txt
python tools/trace_gaps.py "$T" > $O/gaps.txt 2>&1; tail -5 $O/gaps.txt
rm -f "$T"
