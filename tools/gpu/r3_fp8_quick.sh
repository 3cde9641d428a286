#!/bin/bash
# fp8 tests + fp8 / bf16 bench + fp8 kernel table (one box)
set -o pipefail
mkdir -p gpurun_out/fp8q
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py tests/test_model_gpu.py \
  > gpurun_out/fp8q/tests.log 2>&1 || { tail -40 gpurun_out/fp8q/tests.log; exit 1; }
tail -2 gpurun_out/fp8q/tests.log
timeout -k 10 300 python -u bench.py --precision fp8 > gpurun_out/fp8q/fp8.json 2> gpurun_out/fp8q/fp8.err || { tail -20 gpurun_out/fp8q/fp8.err; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/fp8q/bf16.json 2> gpurun_out/fp8q/bf16.err || exit 1
cat gpurun_out/fp8q/fp8.json gpurun_out/fp8q/bf16.json
export TMPDIR=/tmp
timeout -k 10 300 scripts/profile_kernels.sh gpurun_out/fp8q/prof_fp8 -- python bench.py --steps 3 --warmup 4 --precision fp8 \
  > gpurun_out/fp8q/prof_fp8.log 2>&1 || exit 1
python tools/kernel_table.py "$(find gpurun_out/fp8q/prof_fp8 -name 'run_kernel_stats.csv' | head -n 1)" --top 40 --steps 7 \
  > gpurun_out/fp8q/kernel_table_fp8.txt
head -24 gpurun_out/fp8q/kernel_table_fp8.txt
