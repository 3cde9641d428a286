#!/usr/bin/env bash
# The other BASELINE configs on one box: bf16 headline, fp8 (config #5), BERT-large seq 512, reference micro-batch 2x512 (graph).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-configs}
mkdir -p "$O"
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; exit 1; }; echo "$name $(tail -1 "$O/$name.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms/step", "max_mem_gb", d.get("max_mem_gb"))')"; }
run bf16_b256 --steps 20
run fp8_b256 --precision fp8 --steps 20
run large512_b64 --model bert-large-uncased --seq 512 --batch 64 --steps 10 --warmup 3
run ref_micro_b2_s512_graph --batch 2 --seq 512 --graph --steps 50 --warmup 10
