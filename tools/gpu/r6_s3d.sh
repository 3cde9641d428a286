#!/usr/bin/env bash
# Host pacing: bench with the host_issue / host_blocked fields (bf16, fp8), then a cProfile of the bf16 loop.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_s3d}
mkdir -p "$O"
for p in bf16 fp8; do
  timeout -k 10 300 python bench.py --steps 30 --precision $p > "$O/bench_$p.log" 2>&1 || { tail -20 "$O/bench_$p.log"; exit 1; }
  tail -1 "$O/bench_$p.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['value'], d['ms_per_step'], 'issue', d['host_issue_ms'], 'blocked', d['host_blocked_ms'])"
done
timeout -k 10 300 python -m cProfile -o "$O/bench_bf16.prof" bench.py --steps 20 > "$O/cprof_bench.log" 2>&1 || { tail -20 "$O/cprof_bench.log"; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('$O/bench_bf16.prof')
p.sort_stats('tottime').print_stats(45)
" > "$O/cprof_tottime.txt" 2>&1
python3 -c "
import pstats
p = pstats.Stats('$O/bench_bf16.prof')
p.sort_stats('cumulative').print_stats(60)
" > "$O/cprof_cumulative.txt" 2>&1
head -60 "$O/cprof_tottime.txt"
