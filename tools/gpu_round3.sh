#!/usr/bin/env bash
# GPU session 3: kernel tests (incl. native RCCL reducer), bench b64/b256, reference recipe at b256, profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for b in 64 256; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 5 > $O/bench_b$b.log 2>&1 || { tail -20 $O/bench_b$b.log; exit 1; }
  tail -1 $O/bench_b$b.log
done
for attn in sdpa eager; do
  timeout -k 10 600 python tools/ref_recipe_bench.py --batch 256 --steps 10 --warmup 3 --attn $attn > $O/ref256_$attn.log 2>&1 || { tail -20 $O/ref256_$attn.log; exit 1; }
  tail -1 $O/ref256_$attn.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b64 -o run -- python bench.py --batch 64 --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo profiled
