#!/usr/bin/env bash
# Last tree of round 6: the whole GPU suite on the device-assert build, and the fp8 bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3k}
mkdir -p "$O"
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-200
HQ_KERNELS_DEBUG=1 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$O/pytest_debug.log" 2>&1; echo "debug suite rc=$?"; tail -1 "$O/pytest_debug.log"
