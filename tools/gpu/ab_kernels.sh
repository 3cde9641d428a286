#!/usr/bin/env bash
# Same-box interleaved A/B of the headline step: kernel library in ab_old/ vs the in-tree build (static and
# dynamic v3 schedule).  Usage: tools/gpu/ab_kernels.sh <outdir> [rounds]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
R=${2:-3}
mkdir -p "$O"
for r in $(seq 1 $R); do
  for v in old s0 s1; do
    if [ $v = old ]; then E="HQ_KERNELS_DIR=$PWD/ab_old"; else E="HQ_GEMM_SCHED=${v#s}"; fi
    env $E timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v round=$r $(tail -1 "$O/bench_${v}_r$r.log" | cut -c80-175)"
  done
done
