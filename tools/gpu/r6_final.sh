#!/usr/bin/env bash
# Round-6 final tree: whole GPU suite (release), smoke(), headline bench x2, fp8 bench, steady-state bf16 kernel
# table, then the whole GPU suite against the device-assert library.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_final}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
for r in 1 2; do
  timeout -k 10 300 python bench.py > "$O/bench_r$r.log" 2>&1 || { tail -20 "$O/bench_r$r.log"; exit 1; }
  tail -1 "$O/bench_r$r.log" | cut -c1-250
done
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-250
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
T=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_bf16.txt" 2>&1
head -24 "$O/steady_bf16.txt"; tail -2 "$O/steady_bf16.txt"
rm -f "$T"
HQ_KERNELS_DEBUG=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$O/pytest_debug.log" 2>&1; echo "debug suite rc=$?"; tail -3 "$O/pytest_debug.log"
