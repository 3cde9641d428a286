#!/usr/bin/env bash
# memory + throughput sweep: BERT-base seq 384 and BERT-large seq 512 at several per-GPU batches
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_mem
mkdir -p $O
for b in 64 256 512; do
  timeout -k 10 300 python bench.py --batch $b --steps 6 --warmup 3 > $O/base_b$b.log 2>&1 && echo "base b$b $(tail -1 $O/base_b$b.log)" || { tail -3 $O/base_b$b.log; exit 1; }
done
for b in 64 128 256; do
  timeout -k 10 400 python bench.py --model bert-large-uncased --seq 512 --batch $b --steps 5 --warmup 2 > $O/large_b$b.log 2>&1 && echo "large b$b $(tail -1 $O/large_b$b.log)" || { tail -3 $O/large_b$b.log; exit 1; }
done
