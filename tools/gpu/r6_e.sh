#!/usr/bin/env bash
# Full-line epilogue map in every NT GEMM (bf16 v2 / persistent, fp8 v2 / persistent): GEMM, fp8, store and
# model GPU tests, the headline bench, the fp8 bench and a kernel trace of the bf16 step.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_e
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
  tests/test_store_stress_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py tests/test_gemm_sched_gpu.py \
  > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-200
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-200
tools/gpu/step_prof.sh r6_e/step > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -20 "$O/step/kernel_table.txt"
timeout -k 10 400 python tools/ab_step.py --toggle store_nt_all --rounds 4 > "$O/ab_nt_all.log" 2>&1 || { tail -20 "$O/ab_nt_all.log"; exit 1; }
tail -1 "$O/ab_nt_all.log"
