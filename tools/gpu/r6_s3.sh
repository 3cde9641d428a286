#!/usr/bin/env bash
# Round-6 session 3: the rebuilt tree — smoke(), headline bench, fp8 amax-fold deferral A/B (same box,
# interleaved), whole-step graph A/B, then the GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3}
mkdir -p "$O"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench_r1.log" 2>&1 || { tail -20 "$O/bench_r1.log"; exit 1; }
tail -1 "$O/bench_r1.log" | cut -c1-200
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp8_gpu.py > "$O/pytest_fp8.log" 2>&1 \
  || { tail -40 "$O/pytest_fp8.log"; exit 1; }
tail -1 "$O/pytest_fp8.log"
for r in 1 2; do
  HQ_FP8_FOLD_DEFER=1 timeout -k 10 300 python bench.py --precision fp8 --steps 30 > "$O/fp8_defer_r$r.log" 2>&1 || { tail -20 "$O/fp8_defer_r$r.log"; exit 1; }
  tail -1 "$O/fp8_defer_r$r.log" | cut -c1-120
  HQ_FP8_FOLD_DEFER=0 timeout -k 10 300 python bench.py --precision fp8 --steps 30 > "$O/fp8_imm_r$r.log" 2>&1 || { tail -20 "$O/fp8_imm_r$r.log"; exit 1; }
  tail -1 "$O/fp8_imm_r$r.log" | cut -c1-120
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 > "$O/eager_r$r.log" 2>&1 || { tail -20 "$O/eager_r$r.log"; exit 1; }
  tail -1 "$O/eager_r$r.log" | cut -c1-120
  timeout -k 10 300 python bench.py --steps 30 --graph > "$O/graph_r$r.log" 2>&1 || { tail -20 "$O/graph_r$r.log"; exit 1; }
  tail -1 "$O/graph_r$r.log" | cut -c1-120
done
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
