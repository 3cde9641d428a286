#!/usr/bin/env bash
# QA heads backward without the per-sample scalar staging that only dpre_at used: the whole GPU suite, the bf16
# steady-state kernel table (heads rows), smoke and the headline bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3l}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_bf16" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_bf16.log" 2>&1 || { tail -20 "$O/prof_bf16.log"; exit 1; }
T=$(find "$O/prof_bf16" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 --gaps 8 > "$O/steady_bf16.txt" 2>&1
grep -E "qa_|dpre|TOTAL|SPAN" "$O/steady_bf16.txt"
rm -rf "$O/prof_bf16"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-160
