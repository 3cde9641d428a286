#!/usr/bin/env bash
# Kernel tables of the headline step with the fused out-proj/FFN2 + LayerNorm (HQ_LN_FUSE=1) and without.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-lnfuse_prof}
mkdir -p "$O"
for f in 0 1; do
  HQ_LN_FUSE=$f timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p$f" -o run -- python3 bench.py --steps 5 --warmup 3 > "$O/prof$f.log" 2>&1 || { tail -20 "$O/prof$f.log"; exit 1; }
  S=$(find "$O/p$f" -name 'run_kernel_stats.csv' | head -1)
  python tools/kernel_table.py "$S" --steps 8 > "$O/kernel_table_fuse$f.txt" 2>&1
  echo "== fuse=$f"; grep -E "ln_fwd|gemm_nt3_kernel<1>|gemm_nt3_kernel<7>|gemm_nt2_kernel<1|gemm_nt2_kernel<7|TOTAL" "$O/kernel_table_fuse$f.txt"
done
