#!/usr/bin/env bash
# L2 traffic of the persistent NT GEMM at the BERT shapes (T = 98304): L2→fabric read bytes (FETCH_SIZE),
# write bytes, L2 hit/miss, one pass each (per-block counter limits).  10 launches per shape (tools/gemm_one.py).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5_gemm_l2}
mkdir -p "$O"
for shp in "3072 768 1" "2304 768 1" "768 3072 1" "768 768 1"; do
  set -- $shp
  tag=n$1_k$2_e$3
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$O/$tag/f" -o f -- python3 tools/gemm_one.py 98304 $1 $2 $3 > "$O/$tag.f.log" 2>&1 || { tail -5 "$O/$tag.f.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/$tag/w" -o w -- python3 tools/gemm_one.py 98304 $1 $2 $3 > "$O/$tag.w.log" 2>&1 || { tail -5 "$O/$tag.w.log"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/$tag/h" -o h -- python3 tools/gemm_one.py 98304 $1 $2 $3 > "$O/$tag.h.log" 2>&1 || { tail -5 "$O/$tag.h.log"; exit 1; }
  python tools/pmc_summary.py $(find "$O/$tag" -name '*counter_collection.csv') --match gemm > "$O/$tag.txt"
  echo "== $tag"; grep -E "^==|FETCH|WRITE|TCC_|GRBM" "$O/$tag.txt"
done
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d "$O/dram" -o d -- python3 tools/gemm_one.py 98304 3072 768 1 > "$O/dram.log" 2>&1 && python tools/pmc_summary.py $(find "$O/dram" -name '*counter_collection.csv') --match gemm | tee "$O/dram.txt" || echo "dram pass failed (see dram.log)"
