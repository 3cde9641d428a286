#!/usr/bin/env bash
# A/B: nt3 MFMA-group priority levels per wave row (tools/ab_p3: lagging row 2 / leading 1; tools/ab_p4: the
# reverse) vs production (both rows 1).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_prio2
mkdir -p "$O"
for r in 1 2; do
  for v in prod p3 p4; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_$v; fi
    timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_${v}_r$r.log" 2>&1 || { tail -20 "$O/epi_${v}_r$r.log"; exit 1; }
  done
done
unset HQ_KERNELS_DIR
paste "$O/epi_prod_r2.log" "$O/epi_p3_r2.log" "$O/epi_p4_r2.log" | sed 's/"T": 98304, //g; s/"tflops": [0-9.]*//g' | cut -c1-230
