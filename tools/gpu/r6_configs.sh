#!/usr/bin/env bash
# Other configurations on the final round-6 tree: the reference's literal workload (test_bert.cfg geometry:
# 256 per step as 128 micro-batches of 2, seq 512) merged and as a per-micro-batch loop; seq 512 at 256 per GPU;
# BERT-large seq 512 at 64 per GPU; the fp32 mode at the headline shape.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6_configs
mkdir -p "$O"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; exit 1; }
        echo "$name $(tail -1 "$O/$name.log" | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*')"; }
run ref_merged --batch 256 --seq 512 --batch_split 128 --steps 10 --warmup 2
run ref_loop --batch 256 --seq 512 --batch_split 128 --merge off --steps 4 --warmup 1
run seq512 --seq 512 --steps 10 --warmup 3
run large512 --model bert-large-uncased --seq 512 --batch 64 --steps 10 --warmup 3
run large512_fp8 --model bert-large-uncased --seq 512 --batch 64 --precision fp8 --steps 10 --warmup 3
