#!/usr/bin/env bash
# Round-6 first check: the new GPU tests, the whole GPU suite, smoke(), the headline bench and a kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_start
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "sort_ids or embedding" tests/test_fp8_gpu.py::test_gemm_fp8_gelud_bf16_gelu_prime_with_q8 \
  tests/test_model_gpu.py::test_ln_guard_kernel_matches_cpu_rule tests/test_reducer_gpu.py::test_fingerprint_kernel_equals_host \
  tests/test_reducer_gpu.py::test_torchrun_world1_runs_the_n_rank_path tests/test_store_stress_gpu.py::test_embedding_bwd_repeatable \
  > "$O/pytest_new.log" 2>&1 || { tail -60 "$O/pytest_new.log"; exit 1; }
tail -2 "$O/pytest_new.log"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
tools/gpu/step_prof.sh r6_start/step > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -40 "$O/step/kernel_table.txt"
