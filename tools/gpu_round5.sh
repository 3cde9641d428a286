#!/usr/bin/env bash
# GPU session 5: GEMM kernel tests + microbench vs hipBLASLt (LDS-staged epilogue).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -x -q > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 1; }
tail -2 $O/pytest_gemm.log
timeout -k 10 400 python tools/gemm_nt_bench.py > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
cat $O/gemm_bench.log
