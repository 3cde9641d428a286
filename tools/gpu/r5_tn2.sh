#!/usr/bin/env bash
# Lockstep weight-gradient kernel: bitwise test against the alternating-row kernel, then timing per shape.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5_tn2}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "tn" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
TN_VARIANTS=${TN_VARIANTS:-5,1} timeout -k 10 300 python tools/tn_variant_bench.py 9 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.log"
