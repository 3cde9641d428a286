#!/usr/bin/env bash
# store-stress determinism, the full GPU suite, then the fp8 convergence pair
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r4_check2
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_store_stress_gpu.py > "$O/stress.log" 2>&1 \
  || { tail -30 "$O/stress.log"; exit 1; }
tail -1 "$O/stress.log"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
tools/gpu/r4_fp8_conv.sh
