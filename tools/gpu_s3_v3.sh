#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_v3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python tools/ab_step.py --toggle gemm_v2 --rounds 4 --steps 8 > $O/ab.txt 2>&1 && tail -1 $O/ab.txt
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
