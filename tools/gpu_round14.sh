#!/usr/bin/env bash
# Attention v3 kernels: numerics, micro-benchmark, then the b256 bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r14
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "attention" > $O/tests_attn.log 2>&1 || { tail -30 $O/tests_attn.log; exit 1; }
tail -2 $O/tests_attn.log
timeout -k 10 300 python tools/attn_bench.py --B 256 > $O/attn_b256.log 2>&1 && cat $O/attn_b256.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
