#!/usr/bin/env bash
# Per-kernel PMC counters over the headline bench step (2 timed + 1 warmup step), two passes within the
# per-block counter limits (8 SQ / 2 GRBM); summary with MFMA busy, VALU and LDS per MFMA.
# Usage: tools/gpu/step_pmc.sh <outdir> [bench args]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-step_pmc}
shift || true
mkdir -p "$O"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d "$O/a" -o a -- python3 bench.py --steps 2 --warmup 1 "$@" > "$O/a.log" 2>&1 || { tail -20 "$O/a.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$O/b" -o b -- python3 bench.py --steps 2 --warmup 1 "$@" > "$O/b.log" 2>&1 || { tail -20 "$O/b.log"; exit 1; }
python tools/pmc_summary.py $(find "$O/a" -name '*counter_collection.csv') $(find "$O/b" -name '*counter_collection.csv') --match '_kernel' > "$O/summary.txt" 2>&1
grep -E "^==|mfma_busy|VALU / MFMA|LDS / MFMA|lds_conflict" "$O/summary.txt" | head -120
