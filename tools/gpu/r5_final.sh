#!/usr/bin/env bash
# Round-5 final check: full GPU suite, smoke(), the driver's default bench, a kernel trace of the headline
# step, the fp8 bench, and the per-kernel PMC of the step.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_final
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-400
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-250
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table.txt" 2>&1
head -16 "$O/kernel_table.txt"
tools/gpu/step_pmc.sh r5_final/pmc > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
grep -E "^==|mfma_busy" gpurun_out/r5_final/pmc/summary.txt | paste - - | head -20
