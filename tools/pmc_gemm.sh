#!/usr/bin/env bash
# PMC counters of the MFMA NT GEMM on one BERT shape (two passes: SQ core, LDS/memory).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/pmc_gemm
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/a -o a -- python tools/gemm_one.py 98304 3072 768 1 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/b -o b -- python tools/gemm_one.py 98304 3072 768 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python tools/pmc_summary.py $O/a/a_counter_collection.csv $O/b/b_counter_collection.csv --match gemm_nt
