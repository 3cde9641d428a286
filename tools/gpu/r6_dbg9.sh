#!/usr/bin/env bash
# Embedding-gradient zero-fill as an own kernel (no hipMemsetAsync node in the step graph): the synced graph
# divergence, embedding / graph / merge tests.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg9
mkdir -p "$O"
run() { timeout -k 10 200 env "$@" python tools/graph_losses.py > "$O/$1_$2.log" 2>&1; echo "$* rc=$? $(tail -1 "$O/$1_$2.log" | cut -c150-420)"; }
run HQ_SYNC_PROXY=1 X=1
run HQ_KERNELS_DEBUG=1 X=2
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_graph_gpu.py \
  tests/test_merge_gpu.py tests/test_kernels_gpu.py tests/test_f32_ops_gpu.py > "$O/pytest.log" 2>&1; echo "pytest rc=$?"; tail -2 "$O/pytest.log"
