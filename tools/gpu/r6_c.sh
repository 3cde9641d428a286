#!/usr/bin/env bash
# fp32 heads + fold fix: targeted tests and the fp32 step profile; then the whole GPU suite and bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_c
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_f32_ops_gpu.py tests/test_heads_gpu.py tests/test_fp32_gpu.py > "$O/pytest.log" 2>&1 || { tail -60 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 300 python bench.py --precision fp32 --batch 64 --steps 5 --warmup 2 > "$O/bench_fp32.log" 2>&1 || { tail -20 "$O/bench_fp32.log"; exit 1; }
tail -1 "$O/bench_fp32.log" | cut -c1-300
tools/gpu/step_prof.sh r6_c/step_fp32 --precision fp32 --batch 64 > /dev/null 2>&1 || { echo "fp32 profile failed"; exit 1; }
python tools/kernel_table.py "$O/step_fp32/run_kernel_stats.csv" --steps 8 --top 60 > "$O/step_fp32/kernel_table.txt"
head -45 "$O/step_fp32/kernel_table.txt"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-200
