#!/usr/bin/env bash
# Final-tree validation of session 3: whole GPU suite (release), smoke(), headline bench x2, --graph, fp8,
# --force_reducer (1-rank RCCL path), the bf16 step's idle-gap table, then the whole suite on the device-assert build.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3_final2}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
for r in 1 2; do
  timeout -k 10 300 python bench.py > "$O/bench_r$r.log" 2>&1 || { tail -20 "$O/bench_r$r.log"; exit 1; }
  tail -1 "$O/bench_r$r.log" | cut -c1-200
done
timeout -k 10 300 python bench.py --graph > "$O/bench_graph.log" 2>&1 || { tail -20 "$O/bench_graph.log"; exit 1; }
tail -1 "$O/bench_graph.log" | cut -c1-200
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-200
timeout -k 10 300 python bench.py --force_reducer --steps 10 > "$O/bench_force_reducer.log" 2>&1 || { tail -20 "$O/bench_force_reducer.log"; exit 1; }
tail -1 "$O/bench_force_reducer.log" | cut -c1-200
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_bf16" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_bf16.log" 2>&1 || { tail -20 "$O/prof_bf16.log"; exit 1; }
T=$(find "$O/prof_bf16" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 --gaps 12 > "$O/steady_bf16.txt" 2>&1
tail -16 "$O/steady_bf16.txt"
rm -f "$T"
HQ_KERNELS_DEBUG=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$O/pytest_debug.log" 2>&1; echo "debug suite rc=$?"; tail -3 "$O/pytest_debug.log"
