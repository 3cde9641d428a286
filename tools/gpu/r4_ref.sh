#!/usr/bin/env bash
# The reference's literal workload (config/test_bert.cfg geometry: 256 per GPU step as 128 micro-batches of 2,
# seq 512): exact-objective merged pass (default) vs the per-micro-batch loop (--merge off), one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r4_refworkload
mkdir -p "$O"
timeout -k 10 300 python bench.py --batch 256 --seq 512 --batch_split 128 --steps 10 --warmup 2 > "$O/merged.log" 2>&1 \
  || { tail -20 "$O/merged.log"; exit 1; }
tail -1 "$O/merged.log" | cut -c1-300
timeout -k 10 400 python bench.py --batch 256 --seq 512 --batch_split 128 --merge off --steps 4 --warmup 1 > "$O/loop.log" 2>&1 \
  || { tail -20 "$O/loop.log"; exit 1; }
tail -1 "$O/loop.log" | cut -c1-300
