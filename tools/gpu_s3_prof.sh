#!/usr/bin/env bash
# Session 3: attention PMC at the bench shape + per-kernel stats of the b256 bench step + epilogue costs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/s3_prof
mkdir -p $O
timeout -k 10 300 python tools/attn_bench.py --B 256 > $O/attn_b256.txt 2>&1 && cat $O/attn_b256.txt
timeout -k 10 300 python tools/gemm_epi_bench.py > $O/gemm_epi.txt 2>&1 && cat $O/gemm_epi.txt
bash tools/pmc_attn2.sh > $O/pmc_attn.txt 2>&1 || { tail -20 $O/pmc_attn.txt; exit 1; }
cat $O/pmc_attn.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
S=$(find $O/prof -name 'run_kernel_stats.csv' | head -1)
python tools/kernel_table.py "$S" > $O/kernel_table.txt 2>&1; cat $O/kernel_table.txt
