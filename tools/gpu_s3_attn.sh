#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_attn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for c in 0 1 0 1; do
  HQ_ATTN_CHUNK=$c timeout -k 10 120 python tools/attn_bench.py --B 256 > $O/bench_chunk$c.txt 2>&1 && echo "chunk=$c $(grep -v amdgpu $O/bench_chunk$c.txt | tr '\n' ' ')"
done
