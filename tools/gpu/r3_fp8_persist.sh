#!/bin/bash
# persistent fp8 GEMM: correctness (both forms) then v2-vs-persistent timing on the step shapes
set -o pipefail
mkdir -p gpurun_out/fp8p
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py \
  > gpurun_out/fp8p/tests.log 2>&1 || { tail -40 gpurun_out/fp8p/tests.log; exit 1; }
tail -2 gpurun_out/fp8p/tests.log
timeout -k 10 300 python -u tools/fp8_lab/fp8_variant_bench.py > gpurun_out/fp8p/variant_bench.txt 2>&1 || { cat gpurun_out/fp8p/variant_bench.txt; exit 1; }
cat gpurun_out/fp8p/variant_bench.txt
