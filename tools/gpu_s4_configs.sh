#!/usr/bin/env bash
# Session-4 numbers for the BASELINE configs beyond the headline: fp8 (#5), BERT-large seq 512 (#4), b64 / b512.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s4_cfg
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }; echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["max_mem_gb"])')"; }
run base_b256 
run fp8_b256 --precision fp8
run base_b64 --batch 64
run base_b512 --batch 512 --steps 10
run large512_b64 --model bert-large-uncased --seq 512 --batch 64
run large512_b256 --model bert-large-uncased --seq 512 --batch 256 --steps 6 --warmup 3
