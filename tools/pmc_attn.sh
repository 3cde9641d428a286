set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc/a -o a -- python tools/attn_bench.py --B 64 > gpurun_out/pmc/a.log 2>&1 || { tail -20 gpurun_out/pmc/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/b -o b -- python tools/attn_bench.py --B 64 > gpurun_out/pmc/b.log 2>&1 || { tail -20 gpurun_out/pmc/b.log; exit 1; }
find gpurun_out/pmc -name "*counter_collection.csv" | head
