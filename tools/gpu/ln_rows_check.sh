#!/usr/bin/env bash
# Multi-row LayerNorm forward everywhere (bf16, fp8 e4m3-output and z-in variants): full GPU suite, the
# headline bench, the fp8 bench alternating HQ_LN_RPW=1 / 2 twice, and a kernel-trace of the default.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-ln_rows}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
j() { tail -1 "$1" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 200 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
echo "bf16 $(j "$O/bench.log")"
for r in 1 2; do
  for v in 1 2; do
    HQ_LN_RPW=$v timeout -k 10 200 python bench.py --precision fp8 --steps 20 > "$O/fp8_rpw$v.$r.log" 2>&1 || { tail -20 "$O/fp8_rpw$v.$r.log"; exit 1; }
    echo "fp8 rpw=$v round $r $(j "$O/fp8_rpw$v.$r.log")"
  done
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
cp "$S" "$O/run_kernel_stats.csv"
python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table.txt" 2>&1; head -16 "$O/kernel_table.txt"
