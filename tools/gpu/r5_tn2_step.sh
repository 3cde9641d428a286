#!/usr/bin/env bash
# Lockstep weight-gradient kernel: bitwise tests, per-shape timing, and the full bench step with the kernel
# toggled in process (tools/ab_step.py --toggle tn_lockstep).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5_tn2_step}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "tn" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python tools/tn_variant_bench.py 9 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
cat "$O/bench.log"
timeout -k 10 500 python tools/ab_step.py --toggle ${TOGGLE:-tn_auto} --rounds 4 --steps 8 > "$O/ab_step.log" 2>&1 || { tail -20 "$O/ab_step.log"; exit 1; }
tail -4 "$O/ab_step.log"
