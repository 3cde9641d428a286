#!/usr/bin/env bash
# GPU session 7: tests (new dropout hash), tune hipBLASLt for the b256 shapes, bench after tuning.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r7
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
HQ_GEMM=blas HQ_TUNABLEOP=tune HQ_TUNABLEOP_FILE=$O/tuned_blas.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
  timeout -k 10 900 python bench.py --steps 2 --warmup 1 > $O/tune_blas.log 2>&1 || { tail -20 $O/tune_blas.log; exit 1; }
HQ_TUNABLEOP=tune HQ_TUNABLEOP_FILE=$O/tuned_auto.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
  timeout -k 10 900 python bench.py --steps 2 --warmup 1 > $O/tune_auto.log 2>&1 || { tail -20 $O/tune_auto.log; exit 1; }
ls -la $O
wc -l $O/*.csv
