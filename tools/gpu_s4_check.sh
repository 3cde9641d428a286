#!/usr/bin/env bash
# Session-4 sanity on a fresh box: GPU tests, smoke, default bench, kernel-stats profile at b256.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/s4_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
S=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
python tools/kernel_table.py "$S" --steps 8 > $O/kernel_table.txt 2>&1; cat $O/kernel_table.txt
