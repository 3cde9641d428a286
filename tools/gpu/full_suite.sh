#!/bin/bash
# Whole GPU suite + smoke() + one headline bench, each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/full/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 \
  || { tail -30 gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { tail -20 gpurun_out/full/bench.err; exit 1; }
cat gpurun_out/full/bench.json
timeout -k 10 300 python -u bench.py --precision fp8 > gpurun_out/full/bench_fp8.json 2> gpurun_out/full/bench_fp8.err \
  || { tail -20 gpurun_out/full/bench_fp8.err; exit 1; }
cat gpurun_out/full/bench_fp8.json
export TMPDIR=/tmp
timeout -k 10 300 scripts/profile_kernels.sh gpurun_out/full/prof_fp8 -- python bench.py --steps 3 --warmup 4 --precision fp8 \
  > gpurun_out/full/prof_fp8.log 2>&1 || exit 1
python tools/kernel_table.py "$(find gpurun_out/full/prof_fp8 -name 'run_kernel_stats.csv' | head -n 1)" --top 40 --steps 7 \
  > gpurun_out/full/kernel_table_fp8.txt
head -24 gpurun_out/full/kernel_table_fp8.txt
