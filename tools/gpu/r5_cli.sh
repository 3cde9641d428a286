#!/usr/bin/env bash
# fp32 GPU mode tests + the drop-in CLI (train bf16 / fp8 / fp32 -> validate) on the GPU.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_cli
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp32_gpu.py > "$O/pytest_fp32.log" 2>&1
echo "fp32 tests rc=$? $(tail -1 $O/pytest_fp32.log)"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_cli_gpu.py > "$O/pytest_cli.log" 2>&1
echo "cli tests rc=$? $(tail -1 $O/pytest_cli.log)"
