#!/bin/bash
# epilogue store-data experiment: in-tree lib vs tools/ab_so (pad) vs tools/ab_so2 (keep-alive)
set -o pipefail
mkdir -p gpurun_out
for v in "" tools/ab_so tools/ab_so2; do
  echo "== lib ${v:-in-tree}" >> gpurun_out/epi_var.log
  if [ -n "$v" ]; then export HQ_KERNELS_DIR=$v; fi
  timeout -k 10 100 python -u tools/gemm_debug_epi.py >> gpurun_out/epi_var.log 2>&1 || exit $?
  timeout -k 10 100 python -u tools/gemm_debug_epi.py 32768 3072 768 >> gpurun_out/epi_var.log 2>&1 || exit $?
done
cut -c1-220 gpurun_out/epi_var.log
