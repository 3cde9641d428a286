#!/usr/bin/env bash
# fp8: gelu' as an 8-bit code between the FFN1 forward and the FFN2 dgrad.  Tests on the new tree, fp8 benches
# interleaved against the previous whole tree (tools/ab_oldtree = git HEAD package + its kernel library), a kernel
# trace of each, and the fp8 convergence check (seed 0) on the new tree.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_gd8
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_store_stress_gpu.py tests/test_model_gpu.py > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for r in 1 2; do
  (cd tools/ab_oldtree && timeout -k 10 300 python bench.py --steps 30 --precision fp8 > "../../$O/bench_old_r$r.log" 2>&1) || { tail -20 "$O/bench_old_r$r.log"; exit 1; }
  echo "old r$r $(tail -1 "$O/bench_old_r$r.log" | grep -o '"value": [0-9.]*')"
  timeout -k 10 300 python bench.py --steps 30 --precision fp8 > "$O/bench_new_r$r.log" 2>&1 || { tail -20 "$O/bench_new_r$r.log"; exit 1; }
  echo "new r$r $(tail -1 "$O/bench_new_r$r.log" | grep -o '"value": [0-9.]*')"
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_new" -o run -- python3 bench.py --steps 5 --warmup 3 --precision fp8 > "$O/prof_new.log" 2>&1 || { tail -20 "$O/prof_new.log"; exit 1; }
python tools/kernel_table.py "$(find "$O/prof_new" -name 'run_kernel_stats.csv' | head -1)" --steps 8 > "$O/kernel_table_new.txt" 2>&1
cd tools/ab_oldtree && timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "../../$O/prof_old" -o run -- python3 bench.py --steps 5 --warmup 3 --precision fp8 > "../../$O/prof_old.log" 2>&1 || { tail -20 "../../$O/prof_old.log"; exit 1; }
cd ../..
python tools/kernel_table.py "$(find "$O/prof_old" -name 'run_kernel_stats.csv' | head -1)" --steps 8 > "$O/kernel_table_old.txt" 2>&1
OUT=r5_gd8/conv SEEDS=0 tools/gpu/r5_fp8_conv.sh
