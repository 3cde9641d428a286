#!/usr/bin/env bash
# GPU session 12: tests (span head, MFMA-path model parity), bench b256/b64, profile b256.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r12
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b256 -o run -- python bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo profiled
