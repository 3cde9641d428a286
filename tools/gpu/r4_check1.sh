#!/usr/bin/env bash
# Round 4 first GPU check: new tests (segment loss, graph shape cap, reducer proof fields, bench refusal),
# the headline bench, the reference workload (128 x 2 at seq 512) merged, and a kernel profile.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r4_check1
mkdir -p "$O"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 && tail -1 "$O/bench.log" | cut -c1-300 || { tail -20 "$O/bench.log"; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_heads_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py tests/test_gemm_sched_gpu.py \
  tests/test_reducer_gpu.py > "$O/pytest_new.log" 2>&1 || { tail -40 "$O/pytest_new.log"; exit 1; }
tail -3 "$O/pytest_new.log"
timeout -k 10 300 python bench.py --batch 256 --seq 512 --batch_split 128 --steps 3 --warmup 1 > "$O/ref_merged.log" 2>&1 && tail -1 "$O/ref_merged.log" | cut -c1-400 || { tail -20 "$O/ref_merged.log"; exit 1; }
tools/gpu/step_prof.sh r4_check1/prof
