#!/usr/bin/env bash
# GPU session 6: kernel tests, GEMM microbench (fast-erf epilogues), bench A/B of GEMM policy.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python tools/gemm_nt_bench.py > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
grep -E "gelu|98304" $O/gemm_bench.log
for mode in blas auto mfma; do
  HQ_GEMM=$mode timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_$mode.log 2>&1 || { tail -20 $O/bench_$mode.log; exit 1; }
  echo $mode; tail -1 $O/bench_$mode.log
done
HQ_GEMM=auto timeout -k 10 400 python bench.py --batch 64 --steps 20 --warmup 5 > $O/bench_auto_b64.log 2>&1 && tail -1 $O/bench_auto_b64.log
