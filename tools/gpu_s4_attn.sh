#!/usr/bin/env bash
# Session-4: validate the attention/LayerNorm-bwd changes (16-B row stores, deferred rescale, wave priority,
# two-row LN-bwd prefetch) and A/B them on the kernel microbenchmarks and the b256 step.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s4_attn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn or layernorm or ln" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for cfg in "0 0" "0 8" "1 8" "2 8"; do
  set -- $cfg
  HQ_ATTN_PRIO=$1 HQ_ATTN_DEFER=$2 timeout -k 10 120 python tools/attn_bench.py --B 256 > $O/attn_p$1_d$2.txt 2>&1 || { tail $O/attn_p$1_d$2.txt; exit 1; }
  echo "prio=$1 defer=$2 $(grep -v amdgpu $O/attn_p$1_d$2.txt | tr '\n' ' ')"
done
timeout -k 10 120 python tools/ln_bench.py > $O/ln.txt 2>&1 && cat $O/ln.txt
for p in 0 1; do
  HQ_ATTN_PRIO=$p timeout -k 10 300 python bench.py > $O/bench_p$p.log 2>&1 || { tail $O/bench_p$p.log; exit 1; }
  echo "prio=$p $(tail -1 $O/bench_p$p.log | cut -c1-200)"
done
