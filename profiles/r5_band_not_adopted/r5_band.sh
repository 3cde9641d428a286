#!/usr/bin/env bash
# Column-band tile order of the persistent NT GEMM: timing per band width, then L2→fabric read bytes at N = 3072.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5_band}
mkdir -p "$O"
timeout -k 10 400 python tools/gemm_band_bench.py > "$O/band.log" 2>&1 || { tail -20 "$O/band.log"; exit 1; }
cat "$O/band.log"
for b in 0 6 4; do
  fl=$(( (1 << 16) | (b << 18) ))
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$O/f$b" -o f -- python3 tools/gemm_one.py 98304 3072 768 1 0 $fl > "$O/f$b.log" 2>&1 || { tail -5 "$O/f$b.log"; exit 1; }
  echo "band $b: $(python tools/pmc_summary.py $(find "$O/f$b" -name '*counter_collection.csv') --match gemm | grep -E 'FETCH|GRBM' | paste -sd' ')"
done
