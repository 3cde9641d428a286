#!/usr/bin/env bash
# colsum first pass with 16-B loads: tests, step A/B vs tools/ab_so (HEAD norm.hip), steady-state kernel table.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_k
mkdir -p "$O"
AB=$PWD/tools/ab_so
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_heads_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_gemm_gpu.py tests/test_fp8_gpu.py \
  > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export HQ_KERNELS_DIR=$AB; else unset HQ_KERNELS_DIR; fi
    timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
unset HQ_KERNELS_DIR
for v in old new; do
  if [ $v = old ]; then export HQ_KERNELS_DIR=$AB; else unset HQ_KERNELS_DIR; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$v" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  T=$(find "$O/prof_$v" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_$v.txt" 2>&1
  rm -f "$T"
  grep -E "colsum|TOTAL|SPAN" "$O/steady_$v.txt"
done
