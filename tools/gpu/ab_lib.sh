#!/usr/bin/env bash
# Same-box A/B: the kernel library in tools/ab_so/ (tools/build_ab_lib.py) vs the in-tree build — GEMM tests on
# the new build, interleaved headline benches, one kernel-trace profile of each.  Usage: tools/gpu/ab_lib.sh <outdir> [rounds] [tests]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_lib}
R=${2:-3}
T=${3:-tests/test_gemm_gpu.py tests/test_gemm_sched_gpu.py}
AB=${AB:-tools/ab_so}   # the "old" library directory
BA=${BENCH_ARGS:-}       # extra bench.py arguments (e.g. --precision fp8)
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in $(seq 1 $R); do
  for v in old new; do
    if [ $v = old ]; then export HQ_KERNELS_DIR=$PWD/$AB; else unset HQ_KERNELS_DIR; fi
    timeout -k 10 300 python bench.py --steps 30 $BA > "$O/bench_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${v}_r$r.log"; exit 1; }
    echo "$v r$r $(tail -1 "$O/bench_${v}_r$r.log" | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*')"
  done
done
unset HQ_KERNELS_DIR
for v in old new; do
  if [ $v = old ]; then export HQ_KERNELS_DIR=$PWD/$AB; else unset HQ_KERNELS_DIR; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run -- python3 bench.py --steps 5 --warmup 3 $BA > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  S=$(find "$O/prof_$v" -name 'run_kernel_stats.csv' | head -1)
  python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table_$v.txt" 2>&1
done
unset HQ_KERNELS_DIR
paste <(head -14 "$O/kernel_table_old.txt" | cut -c1-100) <(head -14 "$O/kernel_table_new.txt" | cut -c60-100)
