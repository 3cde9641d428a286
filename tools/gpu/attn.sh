#!/usr/bin/env bash
# Attention correctness (GPU tests) then the in-process A/B micro-bench.  Usage: tools/gpu/attn.sh <outdir> [pytest -k]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-attn}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${2:-attention}" > "$O/pytest.log" 2>&1 \
  || { tail -60 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 300 python tools/attn_bench.py --B 256 > "$O/attn_b256.log" 2>&1; cat "$O/attn_b256.log"
