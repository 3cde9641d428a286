#!/usr/bin/env bash
# GPU session 10: attention tests + microbench (cheaper fwd dropout), wgrad split sweep, bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r10
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python tools/attn_bench.py --B 64 > $O/attn_b64.log 2>&1 && cat $O/attn_b64.log
timeout -k 10 600 python tools/wgrad_bench.py > $O/wgrad.log 2>&1 && cat $O/wgrad.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
