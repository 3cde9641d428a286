#!/usr/bin/env bash
# A/B: LayerNorm-bwd two-row prefetch (in-tree build) vs one-row prefetch (tools/ab_so/old_ln), microbench + step
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s4_ln
mkdir -p $O
for r in 1 2; do
  for v in new old; do
    D=ml_recipe_distributed_pytorch_amd; [ $v = old ] && D=tools/ab_so/old_ln
    HQ_KERNELS_DIR=$D timeout -k 10 120 python tools/ln_bench.py > $O/ln_${v}_$r.txt 2>&1 || { tail $O/ln_${v}_$r.txt; exit 1; }
    echo "== $v $r"; grep -v amdgpu $O/ln_${v}_$r.txt
  done
done
for v in new old new old; do
  D=ml_recipe_distributed_pytorch_amd; [ $v = old ] && D=tools/ab_so/old_ln
  HQ_KERNELS_DIR=$D timeout -k 10 300 python bench.py > $O/bench_$v.log 2>&1 || { tail $O/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $O/bench_$v.log | cut -c100-200)"
done
HQ_ATTN_PRIO=2 timeout -k 10 300 python bench.py > $O/bench_prio2.log 2>&1 && echo "prio2 $(tail -1 $O/bench_prio2.log | cut -c100-200)"
