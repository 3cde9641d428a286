#!/usr/bin/env bash
# GPU session: tests, headline bench at several per-GPU batches, reference-recipe baseline, rocprof stats.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for b in 64 128 256; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 5 > $O/bench_b$b.log 2>&1 || { tail -20 $O/bench_b$b.log; exit 1; }
  tail -1 $O/bench_b$b.log
done
for attn in eager sdpa; do
  timeout -k 10 400 python tools/ref_recipe_bench.py --batch 64 --attn $attn > $O/ref_$attn.log 2>&1 || { tail -20 $O/ref_$attn.log; exit 1; }
  tail -1 $O/ref_$attn.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b64 -o run -- python bench.py --batch 64 --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof_b64 -name "*kernel_stats.csv" | head -3
