#!/usr/bin/env bash
# fp8 forward with the caller's grad mode (8-bit gelu' code + no bf16 act in steady state): fp8 / model / CLI
# tests, fp8 bench, steady-state fp8 kernel table.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_g
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fp8_gpu.py \
  tests/test_model_gpu.py > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8_r$r.log" 2>&1 || { tail -20 "$O/bench_fp8_r$r.log"; exit 1; }
tail -1 "$O/bench_fp8_r$r.log" | cut -c1-220
done
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_fp8" -o run -- python3 bench.py --precision fp8 --steps 5 --warmup 12 > "$O/prof_fp8.log" 2>&1 || { tail -20 "$O/prof_fp8.log"; exit 1; }
T=$(find "$O/prof_fp8" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_fp8.txt" 2>&1
head -30 "$O/steady_fp8.txt"; tail -2 "$O/steady_fp8.txt"
rm -f "$T"
