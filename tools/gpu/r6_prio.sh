#!/usr/bin/env bash
# A/B of the nt3 MFMA priority schemes (tools/ab_prio1: static prio for the younger wave row, tools/ab_prio2: none)
# against the production per-group s_setprio: epilogue micro-bench and interleaved headline benches.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_prio
mkdir -p "$O"
for r in 1 2; do
  for v in prod prio1 prio2; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_$v; fi
    timeout -k 10 300 python tools/gemm_epi_bench.py > "$O/epi_${v}_r$r.log" 2>&1 || { tail -20 "$O/epi_${v}_r$r.log"; exit 1; }
  done
done
unset HQ_KERNELS_DIR
paste "$O/epi_prod_r2.log" "$O/epi_prio1_r2.log" "$O/epi_prio2_r2.log" | sed 's/"T": 98304, //g' | cut -c1-250
for r in 1 2; do
  for v in prod prio1 prio2; do
    if [ $v = prod ]; then unset HQ_KERNELS_DIR; else export HQ_KERNELS_DIR=$PWD/tools/ab_$v; fi
    timeout -k 10 300 python bench.py --steps 30 > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
  done
done
