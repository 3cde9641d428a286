#!/usr/bin/env bash
# A/B of the full-line epilogue map (HQ_NT3_LINES=1 lab build in tools/ab_lines) against the in-tree library:
# GEMM correctness tests on the lab build, interleaved epilogue micro-bench, interleaved headline benches.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_lines
mkdir -p "$O"
LAB=$PWD/${LAB:-tools/ab_lines}
HQ_KERNELS_DIR=$LAB timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_store_stress_gpu.py > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_prod_r$r.log" 2>&1 || { tail -20 "$O/epi_prod_r$r.log"; exit 1; }
  HQ_KERNELS_DIR=$LAB timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_lines_r$r.log" 2>&1 || { tail -20 "$O/epi_lines_r$r.log"; exit 1; }
done
paste "$O/epi_prod_r1.log" "$O/epi_lines_r1.log" | cut -c1-200
paste "$O/epi_prod_r2.log" "$O/epi_lines_r2.log" | cut -c1-200
for r in 1 2 3; do
  for v in prod lines; do
    if [ $v = lines ]; then export HQ_KERNELS_DIR=$LAB; else unset HQ_KERNELS_DIR; fi
    timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
