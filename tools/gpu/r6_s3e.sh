#!/usr/bin/env bash
# Copy-stream prefetch of the next batch: the new tests, then benches (bf16 x2, fp8) with the host fields, and the
# step-boundary idle gaps of the new bf16 step.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3e}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_graph_gpu.py \
  > "$O/pytest_graph.log" 2>&1 || { tail -30 "$O/pytest_graph.log"; exit 1; }
tail -1 "$O/pytest_graph.log"
for p in bf16 bf16 fp8; do
  timeout -k 10 300 python bench.py --steps 30 --precision $p > "$O/bench_$p.log" 2>&1 || { tail -20 "$O/bench_$p.log"; exit 1; }
  tail -1 "$O/bench_$p.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['value'], d['ms_per_step'], 'issue', d['host_issue_ms'], 'blocked', d['host_blocked_ms'])"
done
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_bf16" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_bf16.log" 2>&1 || { tail -20 "$O/prof_bf16.log"; exit 1; }
T=$(find "$O/prof_bf16" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 --gaps 12 > "$O/gaps_bf16.txt" 2>&1
tail -16 "$O/gaps_bf16.txt"
rm -f "$T"
