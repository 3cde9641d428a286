#!/usr/bin/env bash
# GPU session 9: fp8 probe, attention microbench at B=64, rocprof of the b256 bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r9
mkdir -p $O
timeout -k 10 300 python tools/fp8_probe.py > $O/fp8_probe.log 2>&1; cat $O/fp8_probe.log | tail -8
timeout -k 10 300 python tools/attn_bench.py --B 64 > $O/attn_b64.log 2>&1 && cat $O/attn_b64.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b256 -o run -- python bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo profiled
