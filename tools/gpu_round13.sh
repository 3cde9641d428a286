#!/usr/bin/env bash
# GPU session 13: tests, bench A/B: side-stream wgrad off/on (b256), residual dgrad on MFMA.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r13
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2; do
  HQ_WGRAD_STREAM=0 timeout -k 10 400 python bench.py > $O/bench_s0_$i.log 2>&1 && echo s0 && tail -1 $O/bench_s0_$i.log
  HQ_WGRAD_STREAM=1 timeout -k 10 400 python bench.py > $O/bench_s1_$i.log 2>&1 && echo s1 && tail -1 $O/bench_s1_$i.log
done
HQ_WGRAD_STREAM=1 timeout -k 10 400 python bench.py --batch 64 > $O/bench_s1_b64.log 2>&1 && echo s1b64 && tail -1 $O/bench_s1_b64.log
