#!/usr/bin/env bash
# Store-pattern lab: epilogue row-piece maps, full chip and 24 workgroups.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5_store_lab
mkdir -p "$O"
timeout -k 10 120 tools/lab/store_pattern 98304 3072 256 > "$O/full.log" 2>&1 || { cat "$O/full.log"; exit 1; }
timeout -k 10 120 tools/lab/store_pattern 6144 3072 24 > "$O/small.log" 2>&1 || { cat "$O/small.log"; exit 1; }
cat "$O/full.log" "$O/small.log"
