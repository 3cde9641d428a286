#!/usr/bin/env bash
# Where the persistent NT GEMM's epilogue time goes: the same shapes/epilogues timed with the production library and
# with lab builds that skip the epilogue's global stores (diag1), the GELU math (diag2) or both (diag3).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_epi_diag
mkdir -p "$O"
for r in 1; do
  for v in prod aux2 aux16 aux18 aux17; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_$v; fi
    timeout -k 10 200 python tools/gemm_epi_bench.py > "$O/${v}_r$r.log" 2>&1 || { tail -5 "$O/${v}_r$r.log"; exit 1; }
    echo "== $v r$r"; grep -E '"N": (3072|768|2304)' "$O/${v}_r$r.log" | python -c "import sys,json; [print(d['N'],d['K'],d['epi'],d['us']) for d in map(json.loads, sys.stdin)]" | paste -sd' ' 
  done
done
