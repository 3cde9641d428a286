#!/usr/bin/env bash
# Pipelined-row LayerNorm forward (tests + in-process step A/B) and the full-line epilogue map A/B (r6_lines.sh).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_d
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  > "$O/pytest_kernels.log" 2>&1 || { tail -40 "$O/pytest_kernels.log"; exit 1; }
tail -1 "$O/pytest_kernels.log"
timeout -k 10 400 python tools/ab_step.py --toggle ln_fwd_pipe --rounds 4 > "$O/ab_ln.log" 2>&1 || { tail -20 "$O/ab_ln.log"; exit 1; }
tail -1 "$O/ab_ln.log"
for v in 1 0; do timeout -k 10 120 python tools/ln_bench.py --fwd_variant $v > "$O/ln_bench_v$v.log" 2>&1 || { tail -20 "$O/ln_bench_v$v.log"; exit 1; }; cat "$O/ln_bench_v$v.log"; done
bash tools/gpu/r6_lines.sh
