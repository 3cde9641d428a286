#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_emb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "embedding" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 120 python tools/embed_bench.py > $O/embed.txt 2>&1 && cat $O/embed.txt
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test_model.log 2>&1 || { tail -30 $O/test_model.log; exit 1; }
tail -2 $O/test_model.log
