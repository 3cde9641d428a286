#!/usr/bin/env bash
# Full GPU check after a change: pytest -m gpu, smoke, headline bench eager and graph, 5-step kernel-trace profile.
# Usage: tools/gpu/full_check.sh <outdir>
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-full}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python __graft_entry__.py > "$O/smoke.log" 2>&1 && tail -1 "$O/smoke.log" || exit 1
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 && tail -1 "$O/bench.log" | cut -c1-260 || { tail -20 "$O/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --graph > "$O/bench_graph.log" 2>&1 && tail -1 "$O/bench_graph.log" | cut -c1-260 || { tail -20 "$O/bench_graph.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
cp "$S" "$O/run_kernel_stats.csv"
python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table.txt" 2>&1; head -16 "$O/kernel_table.txt"
