#!/usr/bin/env bash
# TN (wgrad) kernel: numerics, then vs the hipBLASLt split-K path.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2_tn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -k "tn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python tools/wgrad_tn_bench.py > $O/bench.log 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.log; exit $rc
