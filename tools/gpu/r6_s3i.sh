#!/usr/bin/env bash
# QA heads: forward with the pipelined pooled loop + parallel partial fold (production build) against HEAD's heads.hip
# (tools/ab_heads_old) and two backward variants (tools/ab_heads_r1: R1 register double buffer, tools/ab_heads_r3: R3
# unrolled sample loop): heads tests on production, per-kernel steady-state times of all four.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3i}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_heads_gpu.py \
  tests/test_model_gpu.py > "$O/pytest_heads.log" 2>&1 || { tail -30 "$O/pytest_heads.log"; exit 1; }
tail -1 "$O/pytest_heads.log"
for v in prod old r1 r3 nor3 prod; do
  if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=tools/ab_heads_$v; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$v" -o run -- python3 bench.py --steps 5 --warmup 12 > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  T=$(find "$O/prof_$v" -name 'run_kernel_trace.csv' | head -1)
  python tools/trace_steps.py "$T" --last 5 --top 70 > "$O/steady_$v.txt" 2>&1
  echo "$v: $(grep -E 'qa_heads' "$O/steady_$v.txt" | awk '{print $1, $(NF-1)}' | tr '\n' ' ')"
  rm -rf "$O/prof_$v"
done
