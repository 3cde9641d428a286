#!/usr/bin/env bash
# (1) LayerNorm backward at 16 rows per wave (lab library tools/ab_rpw16) vs production 8: LN tests on the lab
# library, then interleaved headline benches; (2) idle-gap tables of the bf16 and fp8 steady state.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3c}
mkdir -p "$O"
HQ_KERNELS_DIR=tools/ab_rpw16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "ln" > "$O/pytest_ln_rpw16.log" 2>&1 || { tail -30 "$O/pytest_ln_rpw16.log"; exit 1; }
tail -1 "$O/pytest_ln_rpw16.log"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 > "$O/prod_r$r.log" 2>&1 || { tail -20 "$O/prod_r$r.log"; exit 1; }
  tail -1 "$O/prod_r$r.log" | cut -c1-110
  HQ_KERNELS_DIR=tools/ab_rpw16 timeout -k 10 300 python bench.py --steps 30 > "$O/rpw16_r$r.log" 2>&1 || { tail -20 "$O/rpw16_r$r.log"; exit 1; }
  tail -1 "$O/rpw16_r$r.log" | cut -c1-110
done
for p in bf16 fp8; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$p" -o run -- python3 bench.py --steps 5 --warmup 12 --precision $p > "$O/prof_$p.log" 2>&1 || { tail -20 "$O/prof_$p.log"; exit 1; }
  T=$(find "$O/prof_$p" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 --gaps 25 > "$O/gaps_$p.txt" 2>&1
  tail -28 "$O/gaps_$p.txt"
  rm -f "$T"
done
