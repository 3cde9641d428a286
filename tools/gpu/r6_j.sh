#!/usr/bin/env bash
# Release library: graph tests first (the debug-build run failed test_graph_replay_matches_eager), then the
# whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_j
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_graph_gpu.py \
  > "$O/pytest_graph.log" 2>&1; echo "graph tests rc=$?"; grep -E "PASSED|FAILED|ERROR" "$O/pytest_graph.log" | head -20
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1; echo "suite rc=$?"
tail -5 "$O/pytest_gpu.log"
