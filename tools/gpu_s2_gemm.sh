#!/usr/bin/env bash
# GEMM v2: numerics + race screen, lab ablations, then v2 / v1 / hipBLASLt on the BERT shapes, then the bench.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2_gemm
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 tools/gemm_lab/gemm_lab > $O/lab.log 2>&1 || { cat $O/lab.log; exit 1; }
timeout -k 10 400 python tools/gemm_nt_bench.py > $O/bench_nt.log 2>&1 || { cat $O/bench_nt.log; exit 1; }
grep -v amdgpu.ids $O/bench_nt.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 && tail -1 $O/bench.log
