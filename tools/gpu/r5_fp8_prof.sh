#!/usr/bin/env bash
# fp8 step: bench (fp8, fp8 with bf16 dgrads) and a kernel trace of the fp8 step.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_fp8_prof
mkdir -p "$O"
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-220
timeout -k 10 300 python bench.py --precision fp8 --fp8_dgrad 0 > "$O/bench_fp8_dgrad0.log" 2>&1 || { tail -20 "$O/bench_fp8_dgrad0.log"; exit 1; }
tail -1 "$O/bench_fp8_dgrad0.log" | cut -c1-220
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --precision fp8 --steps 10 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python tools/kernel_table.py "$S" --steps 13 > "$O/kernel_table.txt" 2>&1
head -40 "$O/kernel_table.txt"
