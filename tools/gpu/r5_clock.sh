#!/usr/bin/env bash
# Shader clock under load: GRBM_GUI_ACTIVE per dispatch over its wall time, for the MFMA peak loop (no memory
# traffic) and the production GEMMs at the headline shapes.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_clock
mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d "$O/peak" -o run -- tools/mfma_peak/mfma_peak > "$O/peak.log" 2>&1 || { tail -20 "$O/peak.log"; exit 1; }
python tools/clock_summary.py "$O/peak" > "$O/peak_clock.txt" && cat "$O/peak_clock.txt"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d "$O/gemm" -o run -- python3 tools/gemm_epi_bench.py > "$O/gemm.log" 2>&1 || { tail -20 "$O/gemm.log"; exit 1; }
python tools/clock_summary.py "$O/gemm" --match gemm > "$O/gemm_clock.txt" && cat "$O/gemm_clock.txt"
