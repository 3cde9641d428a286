#!/usr/bin/env bash
# GPU session 4: GEMM kernel tests + microbench vs hipBLASLt, then TunableOp tuning for b256 shapes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -x -q > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 1; }
tail -2 $O/pytest_gemm.log
timeout -k 10 400 python tools/gemm_nt_bench.py > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
cat $O/gemm_bench.log
export HQ_TUNABLEOP=tune HQ_TUNABLEOP_FILE=$O/tuned.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
timeout -k 10 900 python bench.py --batch 256 --steps 2 --warmup 1 > $O/tune_b256.log 2>&1 || { tail -20 $O/tune_b256.log; exit 1; }
ls -la $O
