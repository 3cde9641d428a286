#!/usr/bin/env bash
# Per-kernel HIP time of any training / bench command (SURVEY §5.1 "--profile with a rocprofv3 wrapper"):
# rocprofv3 kernel trace + stats into OUT_DIR, then a short table of the top kernels by total time.
#
#   scripts/profile_kernels.sh OUT_DIR -- python bench.py --steps 5 --warmup 3
#   scripts/profile_kernels.sh OUT_DIR -- python modules/train.py -c config/test_bert.cfg --local_rank 0 --profile
#
# The program must follow `--` directly (no env/bash -c wrappers: the profiler's preload must not exec).
set -eo pipefail
out="${1:?usage: profile_kernels.sh OUT_DIR -- COMMAND ...}"
shift
[ "$1" = "--" ] && shift
here="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$out"
export TMPDIR="${TMPDIR:-/tmp}"
rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- "$@"
stats="$(find "$out" -name 'run_kernel_stats.csv' | head -n 1)"
python "$here/tools/kernel_table.py" "$stats" --top 25 | tee "$out/kernel_table.txt"
