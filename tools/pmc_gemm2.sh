#!/usr/bin/env bash
# PMC counters of GEMM v2 (and v1 for contrast) on a long-K and a short-K BERT shape.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/pmc_gemm2
mkdir -p $O
run() {  # tag variant T N K
  HQ_GEMM_VARIANT=$2 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/$1a -o a -- python tools/gemm_one.py $3 $4 $5 0 > $O/$1a.log 2>&1 || return 1
  HQ_GEMM_VARIANT=$2 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/$1b -o b -- python tools/gemm_one.py $3 $4 $5 0 > $O/$1b.log 2>&1 || return 1
  HQ_GEMM_VARIANT=$2 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/$1c -o c -- python tools/gemm_one.py $3 $4 $5 0 > $O/$1c.log 2>&1 || return 1
  echo "######## $1 (variant $2, T=$3 N=$4 K=$5)"
  python tools/pmc_summary.py $O/$1a/a_counter_collection.csv $O/$1b/b_counter_collection.csv $O/$1c/c_counter_collection.csv --match gemm_nt
}
run longk 0 98304 768 3072 && run shortk 0 98304 3072 768 && run shortk_v1 1 98304 3072 768
