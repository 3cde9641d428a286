#!/usr/bin/env bash
# fp8 vs bf16 convergence on the learnable synthetic NQ task (tools/fp8_convergence.py), same seed / order.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r4_fp8_conv
mkdir -p "$O"
for p in bf16 fp8; do
  timeout -k 10 500 python -u tools/fp8_convergence.py --precision $p --out "$O" > "$O/run_$p.log" 2>&1 \
    || { tail -30 "$O/run_$p.log"; exit 1; }
  tail -1 "$O/run_$p.log" | cut -c1-600
done
