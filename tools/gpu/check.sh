#!/usr/bin/env bash
# One GPU-box session: pytest -m gpu (+ optional -k filter), smoke, the headline bench and the forced
# native-reducer bench, an attention micro-bench.  Usage: tools/gpu/check.sh <outdir> [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
K=${2:-}
mkdir -p "$O"
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${KARG[@]}" > "$O/pytest_gpu.log" 2>&1 \
  || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python __graft_entry__.py > "$O/smoke.log" 2>&1 && cat "$O/smoke.log" || exit 1
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 && tail -1 "$O/bench.log" || { tail -20 "$O/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --force_reducer > "$O/bench_force_reducer.log" 2>&1 && tail -1 "$O/bench_force_reducer.log" || { tail -20 "$O/bench_force_reducer.log"; exit 1; }
timeout -k 10 300 python tools/attn_bench.py --B 256 > "$O/attn_b256.log" 2>&1 && cat "$O/attn_b256.log"
