#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3_ab
mkdir -p $O
for t in "fwd_mfma=qkv" "fwd_mfma=qkv,out,ffn2" "fwd_mfma=qkv,out"; do
  timeout -k 10 300 python tools/ab_step.py --toggle "$t" --rounds 4 --steps 8 > "$O/ab_$t.txt" 2>&1 || { tail -20 "$O/ab_$t.txt"; exit 1; }
  tail -3 "$O/ab_$t.txt"
done
