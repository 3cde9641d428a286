#!/usr/bin/env bash
# Same-box A/B of the v3 tile schedule in the headline step (interleaved) + uncontended GEMM timings.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-sched_step}
mkdir -p "$O"
timeout -k 10 300 python -u tools/gemm_contention_bench.py --rounds 21 --hogs 0 > "$O/uncontended.log" 2>&1 || { tail -30 "$O/uncontended.log"; exit 1; }
cat "$O/uncontended.log" | cut -c1-200
for r in 1 2 3; do for s in 0 1; do
  HQ_GEMM_SCHED=$s timeout -k 10 300 python bench.py --steps 30 > "$O/bench_s${s}_r$r.log" 2>&1 || { tail -20 "$O/bench_s${s}_r$r.log"; exit 1; }
  echo "sched=$s round=$r $(tail -1 "$O/bench_s${s}_r$r.log" | cut -c80-170)"
done; done
