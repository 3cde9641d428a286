#!/usr/bin/env bash
# Full GPU test suite, default bench, b64 bench, then a kernel profile of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/s2_step
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log || exit 1
timeout -k 10 600 python bench.py --batch 64 > $O/bench_b64.log 2>&1 && tail -1 $O/bench_b64.log || exit 1
timeout -k 10 400 scripts/profile_kernels.sh $O/prof -- python bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 && tail -27 $O/prof.log
