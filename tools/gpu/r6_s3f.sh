#!/usr/bin/env bash
# Same-box A/B of the copy-stream prefetch (HQ_BENCH_PREFETCH=1 default vs 0: copies on the compute stream), bf16
# and fp8, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3f}
mkdir -p "$O"
for r in 1 2; do
  for p in bf16 fp8; do
    for pf in 1 0; do
      HQ_BENCH_PREFETCH=$pf timeout -k 10 300 python bench.py --steps 30 --precision $p > "$O/${p}_pf${pf}_r$r.log" 2>&1 || { tail -20 "$O/${p}_pf${pf}_r$r.log"; exit 1; }
      tail -1 "$O/${p}_pf${pf}_r$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p pf$pf r$r', d['value'], d['ms_per_step'], 'blocked', d['host_blocked_ms'])"
    done
  done
done
