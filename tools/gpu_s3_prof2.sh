#!/usr/bin/env bash
# current per-kernel table + idle-gap accounting of the b256 bench step
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/s3_prof2
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
S=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
T=$(find $O/prof -name 'run_kernel_trace.csv' | head -1)
python tools/kernel_table.py "$S" --steps 11 > $O/kernel_table.txt 2>&1; cat $O/kernel_table.txt
python tools/trace_gaps.py "$T" > $O/gaps.txt 2>&1; cat $O/gaps.txt
