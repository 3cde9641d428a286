#!/usr/bin/env bash
# Multi-row LayerNorm forward (dropout + residual variant): rows per wave HQ_LN_RPW = 1 (the one-row
# form) / 2 / 4.  LN GPU tests, the headline bench alternating the three twice on one box, then a
# short kernel-trace per setting for the per-kernel time.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ln_rpw}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_ln_fuse_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for r in 1 2; do
  for v in 1 2 4; do
    HQ_LN_RPW=$v timeout -k 10 200 python bench.py > "$O/bench_rpw$v.$r.log" 2>&1 || { tail -20 "$O/bench_rpw$v.$r.log"; exit 1; }
    echo "rpw=$v round $r $(tail -1 "$O/bench_rpw$v.$r.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for v in 1 2 4; do
  HQ_LN_RPW=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$v" -o run -- python3 bench.py --steps 3 --warmup 2 > "$O/prof$v.log" 2>&1 || { tail -20 "$O/prof$v.log"; exit 1; }
  S=$(find "$O/prof$v" -name 'run_kernel_stats.csv' | head -1)
  python tools/kernel_table.py "$S" --steps 5 > "$O/kernel_table$v.txt" 2>&1
  echo "rpw=$v"; grep -E "ln_fwd|TOTAL" "$O/kernel_table$v.txt"
done
