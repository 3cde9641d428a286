#!/usr/bin/env bash
# P23 wait for both wave rows (latent row-0 RAW on LDS-DMA rows): GEMM tests, per-GEMM and step A/B vs the
# previous kernels (tools/ab_old = HEAD~ gemm.hip / gemm_fp8.hip / gemm_tn.hip).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_race
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_store_stress_gpu.py tests/test_fp8_gpu.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  for v in new old; do
    if [ $v = new ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_old; fi
    timeout -k 10 200 python tools/gemm_epi_bench.py > "$O/gemm_${v}_r$r.log" 2>&1 || { tail -5 "$O/gemm_${v}_r$r.log"; exit 1; }
    echo "== gemm $v r$r"; grep -E '"N": (3072|768|2304)' "$O/gemm_${v}_r$r.log" | python -c "import sys,json; [print(d['N'],d['K'],d['epi'],d['us']) for d in map(json.loads, sys.stdin)]" | paste -sd' '
    timeout -k 10 300 python bench.py > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "== bench $v r$r"; tail -1 "$O/bench_${v}_r$r.log" | cut -c1-200
  done
done
