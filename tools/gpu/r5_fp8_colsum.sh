#!/usr/bin/env bash
# fp8 attention backward: colsum butterfly selects as v_cndmask (no 16-way compare chains). Tests, bench, trace.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_fp8_colsum
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_gpu.py tests/test_kernels_gpu.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python bench.py --precision fp8 > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-220
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --precision fp8 --steps 10 --warmup 3 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
S=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python tools/kernel_table.py "$S" --steps 13 > "$O/kernel_table.txt" 2>&1
head -30 "$O/kernel_table.txt"
