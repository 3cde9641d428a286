#!/usr/bin/env bash
# A/B: s_setprio around the MFMA groups of dQ only (tools/ab_ap2) or dK/dV only (tools/ab_ap4) vs production.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_ap
mkdir -p "$O"
for r in 1 2; do
  for v in prod ap2 ap4; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_$v; fi
    timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn_${v}_r$r.log" 2>&1 || { tail -20 "$O/attn_${v}_r$r.log"; exit 1; }
  done
done
unset HQ_KERNELS_DIR
for v in prod ap2 ap4; do echo "== $v"; grep "round [12]" "$O/attn_${v}_r2.log"; done
