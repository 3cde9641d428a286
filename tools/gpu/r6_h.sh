#!/usr/bin/env bash
# (1) whole-line attention output stores (fwd ctx, dK/dV): kernel tests, attention micro-bench and step A/B vs
# tools/ab_so (HEAD attention.hip); (2) the fp8 grad-mode fix: fp8 / model tests, fp8 bench, steady-state table.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_h
mkdir -p "$O"
AB=$PWD/tools/ab_so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_store_stress_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  HQ_KERNELS_DIR=$AB timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn_old_r$r.log" 2>&1 || { tail -20 "$O/attn_old_r$r.log"; exit 1; }
  timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn_new_r$r.log" 2>&1 || { tail -20 "$O/attn_new_r$r.log"; exit 1; }
done
paste "$O/attn_old_r2.log" "$O/attn_new_r2.log" | cut -c1-220
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export HQ_KERNELS_DIR=$AB; else unset HQ_KERNELS_DIR; fi
    timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
unset HQ_KERNELS_DIR
for r in 1 2; do
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8_r$r.log" 2>&1 || { tail -20 "$O/bench_fp8_r$r.log"; exit 1; }
tail -1 "$O/bench_fp8_r$r.log" | cut -c1-220
done
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_fp8" -o run -- python3 bench.py --precision fp8 --steps 5 --warmup 12 > "$O/prof_fp8.log" 2>&1 || { tail -20 "$O/prof_fp8.log"; exit 1; }
T=$(find "$O/prof_fp8" -name 'run_kernel_trace.csv' | head -1)
python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_fp8.txt" 2>&1
head -30 "$O/steady_fp8.txt"; tail -2 "$O/steady_fp8.txt"
rm -f "$T"
