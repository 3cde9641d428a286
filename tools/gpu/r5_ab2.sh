#!/usr/bin/env bash
# Same-box A/B of tools/ab_old vs the in-tree build on the bf16 AND fp8 benches, plus kernel tables of both
# builds for each precision.  Usage: tools/gpu/r5_ab2.sh <outdir> [tests]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ab2}
T=${2:-tests/test_gemm_gpu.py}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  for prec in bf16 fp8; do
    for v in old new; do
      if [ $v = old ]; then export HQ_KERNELS_DIR=$PWD/tools/ab_old; else unset HQ_KERNELS_DIR; fi
      timeout -k 10 300 python bench.py --steps 30 --precision $prec > "$O/bench_${prec}_${v}_r$r.log" 2>&1 || { tail -20 "$O/bench_${prec}_${v}_r$r.log"; exit 1; }
      echo "$prec $v r$r $(tail -1 "$O/bench_${prec}_${v}_r$r.log" | grep -o '"value": [0-9.]*')"
    done
  done
done
for prec in bf16 fp8; do
  for v in old new; do
    if [ $v = old ]; then export HQ_KERNELS_DIR=$PWD/tools/ab_old; else unset HQ_KERNELS_DIR; fi
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${prec}_$v" -o run -- python3 bench.py --steps 5 --warmup 3 --precision $prec > "$O/prof_${prec}_$v.log" 2>&1 || { tail -20 "$O/prof_${prec}_$v.log"; exit 1; }
    S=$(find "$O/prof_${prec}_$v" -name 'run_kernel_stats.csv' | head -1)
    python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table_${prec}_$v.txt" 2>&1
  done
done
unset HQ_KERNELS_DIR
