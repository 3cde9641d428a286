#!/usr/bin/env bash
# A/B: attention kernels with s_setprio 1 around their MFMA groups (tools/ab_aprio) vs production.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_aprio
mkdir -p "$O"
AB=$PWD/tools/ab_aprio
HQ_KERNELS_DIR=$AB timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "attention" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn_prod_r$r.log" 2>&1 || { tail -20 "$O/attn_prod_r$r.log"; exit 1; }
  HQ_KERNELS_DIR=$AB timeout -k 10 200 python tools/attn_bench.py --rounds 2 > "$O/attn_prio_r$r.log" 2>&1 || { tail -20 "$O/attn_prio_r$r.log"; exit 1; }
done
paste "$O/attn_prod_r2.log" "$O/attn_prio_r2.log" | cut -c1-220
for r in 1 2; do
  for v in prod prio; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$AB; fi
    timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
