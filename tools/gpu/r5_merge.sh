#!/usr/bin/env bash
# GPU merged-segment engine test (exact-objective merge vs accumulation, graphs off/on)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5_merge
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_merge_gpu.py > "$O/pytest.log" 2>&1; rc=$?
tail -15 "$O/pytest.log"
exit $rc
