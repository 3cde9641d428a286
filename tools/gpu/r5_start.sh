#!/usr/bin/env bash
# Round-5 start: new fp32 GPU tests, headline bench + kernel trace of the step on this box (baseline for the round).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_start
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp32_gpu.py > "$O/pytest_fp32.log" 2>&1
echo "fp32 tests rc=$? $(tail -1 $O/pytest_fp32.log)"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
tools/gpu/step_prof.sh r5_start/step > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
head -30 "$O/step/kernel_table.txt"
