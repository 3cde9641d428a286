#!/usr/bin/env bash
# Whole GPU suite against the device-assert kernel library (<pkg>/_debug, HQ_DASSERT bounds / shape checks on).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_dbg
mkdir -p "$O"
HQ_KERNELS_DEBUG=1 timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
