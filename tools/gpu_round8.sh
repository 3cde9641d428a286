#!/usr/bin/env bash
# GPU session 8: attention (prescaled Q, bias-initialised accumulators, new dropout hash) tests and
# microbench; GEMM microbench and bench A/B with the b256 TunableOp results shipped.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r8
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python tools/attn_bench.py --B 256 > $O/attn_b256.log 2>&1 || { tail -20 $O/attn_b256.log; exit 1; }
cat $O/attn_b256.log
timeout -k 10 400 python tools/gemm_nt_bench.py > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
grep -E "98304" $O/gemm_bench.log
for mode in blas auto mfma; do
  HQ_GEMM=$mode timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_$mode.log 2>&1 || { tail -20 $O/bench_$mode.log; exit 1; }
  echo $mode; tail -1 $O/bench_$mode.log
done
