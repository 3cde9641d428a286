#!/usr/bin/env bash
# LayerNorm backward from y (no stored z) vs the z-storing form: full GPU suite, then the headline bench
# alternating HQ_LN_FROM_Y=0 / 1 twice on one box, then a kernel-trace profile of the default.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ln_from_y}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for r in 1 2; do
  for v in 0 1; do
    HQ_LN_FROM_Y=$v timeout -k 10 200 python bench.py > "$O/bench_fromy$v.$r.log" 2>&1 || { tail -20 "$O/bench_fromy$v.$r.log"; exit 1; }
    echo "from_y=$v round $r $(tail -1 "$O/bench_fromy$v.$r.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["max_mem_gb"])')"
  done
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
cp "$S" "$O/run_kernel_stats.csv"
python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table.txt" 2>&1; head -16 "$O/kernel_table.txt"
