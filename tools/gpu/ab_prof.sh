#!/usr/bin/env bash
# Kernel tables of the headline step: in-tree build vs the build in $1 (HQ_KERNELS_DIR), same box.
# Usage: tools/gpu/ab_prof.sh <alt_dir> <outdir> [kernel-name regex]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
ALT=$1; O=gpurun_out/${2:-ab_prof}; RX=${3:-TOTAL}
mkdir -p "$O"
for v in base alt; do
  if [ $v = alt ]; then E="HQ_KERNELS_DIR=$PWD/$ALT"; else E="HQ_AB=base"; fi
  env $E timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$v" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  S=$(find "$O/p_$v" -name 'run_kernel_stats.csv' | head -1)
  python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table_$v.txt" 2>&1
  echo "== $v"; grep -E "$RX|TOTAL" "$O/kernel_table_$v.txt"
done
