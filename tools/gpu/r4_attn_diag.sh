#!/bin/bash
# attention numerics: in-tree lib vs tools/ab_so2 (HEAD attention), then the GEMM A/B (tools/ab_so = HEAD gemm)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/attn_diag.py > gpurun_out/attn_diag_new.log 2>&1 || exit $?
HQ_KERNELS_DIR=tools/ab_so2 timeout -k 10 120 python -u tools/attn_diag.py > gpurun_out/attn_diag_old.log 2>&1 || exit $?
grep ramp gpurun_out/attn_diag_new.log; echo ==; grep ramp gpurun_out/attn_diag_old.log
