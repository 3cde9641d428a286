#!/usr/bin/env bash
# GPU session 11: full GPU tests (fp8 quant/linear/model), bench bf16 (new wgrad splits) and fp8.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r11
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --precision fp8 > $O/bench_fp8.log 2>&1 && tail -1 $O/bench_fp8.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 64 > $O/bench_b64.log 2>&1 && tail -1 $O/bench_b64.log
timeout -k 10 600 python bench.py --model bert-large-uncased --seq 512 --batch 64 --steps 10 --warmup 3 > $O/bench_large512.log 2>&1 && tail -1 $O/bench_large512.log
