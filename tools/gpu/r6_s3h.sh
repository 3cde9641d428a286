#!/usr/bin/env bash
# QA heads with register-double-buffered pooled loops (production) vs HEAD's heads.hip (tools/ab_heads_old):
# heads tests, per-kernel steady-state times of both, interleaved headline benches.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3h}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heads_gpu.py \
  tests/test_model_gpu.py > "$O/pytest_heads.log" 2>&1 || { tail -30 "$O/pytest_heads.log"; exit 1; }
tail -1 "$O/pytest_heads.log"
for v in new old; do
  if [ $v = old ]; then export HQ_KERNELS_DIR=tools/ab_heads_old; else unset HQ_KERNELS_DIR; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$v" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  T=$(find "$O/prof_$v" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_$v.txt" 2>&1
  echo "$v: $(grep -E 'qa_heads' "$O/steady_$v.txt" | tr -s ' ' | cut -d' ' -f1,4 | tr '\n' ' ') $(tail -2 "$O/steady_$v.txt" | tr -s ' ' | tr '\n' ' ')"
  rm -f "$T"
done
unset HQ_KERNELS_DIR
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 > "$O/new_r$r.log" 2>&1 || { tail -20 "$O/new_r$r.log"; exit 1; }
  tail -1 "$O/new_r$r.log" | cut -c1-110
  HQ_KERNELS_DIR=tools/ab_heads_old timeout -k 10 300 python bench.py --steps 30 > "$O/old_r$r.log" 2>&1 || { tail -20 "$O/old_r$r.log"; exit 1; }
  tail -1 "$O/old_r$r.log" | cut -c1-110
done
