#!/usr/bin/env bash
# Lab: the epilogue operand loads of DMUL / RESID from an L2-resident window (HQ_EPI_DIAG=64, results wrong)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_diag64
mkdir -p "$O"
for r in 1 2; do
  timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_prod_r$r.log" 2>&1 || { tail -20 "$O/epi_prod_r$r.log"; exit 1; }
  HQ_KERNELS_DIR=$PWD/tools/ab_diag64 timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_diag_r$r.log" 2>&1 || { tail -20 "$O/epi_diag_r$r.log"; exit 1; }
done
paste "$O/epi_prod_r2.log" "$O/epi_diag_r2.log" | sed 's/"T": 98304, //g' | cut -c1-200
