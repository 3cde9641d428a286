#!/usr/bin/env bash
# Kernel-trace stats + two PMC passes of the v3 attention kernels at B=256, L=384.  Usage: tools/gpu/attn_prof.sh <outdir>
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-attn_prof}
mkdir -p "$O"
ARGS="--B 256 --fwd 3 --bwd 3 --rounds 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python tools/attn_bench.py $ARGS > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
python tools/kernel_table.py $(find "$O/kt" -name '*kernel_stats.csv' | head -1) --steps 1 > "$O/kernel_table.txt" 2>&1; head -12 "$O/kernel_table.txt"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$O/a" -o a -- python tools/attn_bench.py $ARGS > "$O/a.log" 2>&1 || { tail -20 "$O/a.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d "$O/b" -o b -- python tools/attn_bench.py $ARGS > "$O/b.log" 2>&1 || { tail -20 "$O/b.log"; exit 1; }
python tools/pmc_summary.py $(find "$O/a" -name '*counter_collection.csv') $(find "$O/b" -name '*counter_collection.csv') --match attn > "$O/summary.txt" 2>&1
cat "$O/summary.txt"
