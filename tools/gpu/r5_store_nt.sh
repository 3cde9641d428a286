#!/usr/bin/env bash
# Streamed (nt|sc1) epilogue stores: GEMM tests, in-process step A/B, bench, store retirement lab.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_store_nt
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_store_stress_gpu.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 400 python tools/ab_step.py --toggle store_nt --rounds 4 > "$O/ab_store_nt.log" 2>&1 || { tail -20 "$O/ab_store_nt.log"; exit 1; }
cat "$O/ab_store_nt.log"
timeout -k 10 400 python tools/ab_step.py --toggle store_nt_all --rounds 3 > "$O/ab_store_nt_all.log" 2>&1 || { tail -20 "$O/ab_store_nt_all.log"; exit 1; }
cat "$O/ab_store_nt_all.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-200
timeout -k 10 120 tools/lab/store_pattern 98304 3072 256 > "$O/lab_full.log" 2>&1 && tail -1 "$O/lab_full.log"
timeout -k 10 120 tools/lab/store_pattern 6144 3072 24 > "$O/lab_small.log" 2>&1 && tail -1 "$O/lab_small.log"
