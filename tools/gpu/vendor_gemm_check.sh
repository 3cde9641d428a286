#!/usr/bin/env bash
# Kernel-trace the training step at the small / irregular shapes and list any vendor GEMM kernels
# (hipBLASLt "Cijk_" / rocBLAS) that ran: bench --batch 64, the reference micro-batch --batch 2 --seq 512,
# and a dynamically padded batch (--batch 4 --seq 317: M = 1268, not a multiple of 256).
# Usage: tools/gpu/vendor_gemm_check.sh <outdir>
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-vendor_gemm}
mkdir -p "$O"
: > "$O/summary.txt"
for cfg in "64 384" "2 512" "4 317"; do
  set -- $cfg
  tag="b$1_s$2"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$tag" -o run -- \
    python3 bench.py --batch "$1" --seq "$2" --steps 3 --warmup 2 > "$O/$tag.log" 2>&1 || { tail -20 "$O/$tag.log"; exit 1; }
  S=$(find "$O/$tag" -name 'run_kernel_stats.csv' | head -1)
  n=$(grep -ciE 'Cijk_|hipblaslt|rocblas|gemm_kernel|Tensile' "$S" || true)
  echo "$tag vendor_gemm_kernels=$n $(grep '"metric"' "$O/$tag.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("samples_per_s=%s ms_per_step=%s" % (d["value"], d["ms_per_step"]))')" >> "$O/summary.txt"
  grep -iE 'Cijk_|hipblaslt|rocblas|Tensile' "$S" | cut -c1-160 >> "$O/summary.txt" || true
done
cat "$O/summary.txt"
