#!/usr/bin/env bash
# fp8: persistent kernel for the Q8 DMUL too (in-process step A/B), plus the dropout-free dQ priority check.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_i
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "attention" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn.log" 2>&1 || { tail -20 "$O/attn.log"; exit 1; }
grep "round 1" "$O/attn.log"
timeout -k 10 500 python tools/ab_step.py --precision fp8 --toggle fp8_persist --rounds 4 > "$O/ab_fp8_persist.log" 2>&1 || { tail -20 "$O/ab_fp8_persist.log"; exit 1; }
tail -1 "$O/ab_fp8_persist.log"
