#!/usr/bin/env bash
# Kernel traces of the step with the persistent GEMM's epilogue stores default-policy (off) vs streamed (on).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_store_nt_prof
mkdir -p "$O"
for arm in off on; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$arm" -o run -- python3 tools/ab_step.py --toggle store_nt --only $arm --rounds 1 --steps 4 > "$O/$arm.log" 2>&1 || { tail -20 "$O/$arm.log"; exit 1; }
  S=$(find "$O/$arm" -name 'run_kernel_stats.csv' | head -1)
  python tools/kernel_table.py "$S" --steps 10 > "$O/kernel_table_$arm.txt" 2>&1
done
paste <(head -22 "$O/kernel_table_off.txt" | cut -c1-100) <(head -22 "$O/kernel_table_on.txt" | cut -c60-100)
