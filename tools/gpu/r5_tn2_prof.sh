#!/usr/bin/env bash
# Kernel traces of the bench step with the alternating-row (tn 0) and lockstep (tn 1) weight-gradient kernels.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5_tn2_prof}
mkdir -p "$O"
for v in ${TN_ARMS:-5 0}; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run -- python3 tools/bench_variant.py --tn $v -- --steps 5 --warmup 3 > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  python tools/kernel_table.py "$(find "$O/prof_$v" -name 'run_kernel_stats.csv' | head -1)" --steps 8 > "$O/kernel_table_$v.txt" 2>&1
  grep -E "gemm_tn|TOTAL" "$O/kernel_table_$v.txt"
done
for r in 1 2; do
  for v in ${TN_ARMS:-5 0}; do
    timeout -k 10 300 python tools/bench_variant.py --tn $v -- --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "tn$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
