#!/usr/bin/env bash
# Box normalisation for r6_configs: the headline bench and seq 512 back to back on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6_configs/norm
mkdir -p "$O"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; exit 1; }
        echo "$name $(tail -1 "$O/$name.log" | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*')"; }
run headline --steps 20 --warmup 5
run seq512 --seq 512 --steps 10 --warmup 3
run headline2 --steps 20 --warmup 5
