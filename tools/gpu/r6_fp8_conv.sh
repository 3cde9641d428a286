#!/usr/bin/env bash
# fp8 vs bf16 convergence on the learnable synthetic NQ task (tools/fp8_convergence.py): per seed, the same
# init and sample order for both precisions; two seeds show the run-to-run spread.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6_fp8_conv}
mkdir -p "$O"
for s in ${SEEDS:-0 1}; do
  for p in bf16 fp8; do
    timeout -k 10 400 python -u tools/fp8_convergence.py --precision $p --seed $s --steps ${STEPS:-1000} \
      --lr ${LR:-5e-5} --out "$O" > "$O/run_${p}_s$s.log" 2>&1 || { tail -30 "$O/run_${p}_s$s.log"; exit 1; }
    tail -1 "$O/run_${p}_s$s.log" | cut -c1-1500
  done
done
