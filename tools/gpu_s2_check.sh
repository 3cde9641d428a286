#!/usr/bin/env bash
# Session-2 sanity: GPU tests, smoke, default bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
