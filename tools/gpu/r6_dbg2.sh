#!/usr/bin/env bash
# Debug-assert library: test_graph_gpu twice (reproducibility of the step-4 loss mismatch seen in r6_dbg), then
# the rest of the GPU suite past it.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg2
mkdir -p "$O"
for r in 1 2; do
  HQ_KERNELS_DEBUG=1 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py > "$O/graph_r$r.log" 2>&1; echo "graph r$r rc=$?"
  grep -E "PASSED|FAILED|^E .*assert" "$O/graph_r$r.log" | head -12
done
HQ_KERNELS_DEBUG=1 timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_graph_gpu.py > "$O/pytest.log" 2>&1; echo "suite rc=$?"
tail -3 "$O/pytest.log"
