#!/usr/bin/env bash
# Session 3: attention-forward lab variants (prologue-only, v2, persistent v4) + embedding-bwd cost split.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_lab
mkdir -p $O
timeout -k 10 200 bash tools/attn_lab/run.sh 256 > $O/attn_lab.txt 2>&1; cat $O/attn_lab.txt | tail -30
timeout -k 10 120 python tools/embed_bench.py > $O/embed.txt 2>&1 && cat $O/embed.txt
