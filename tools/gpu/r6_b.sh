#!/usr/bin/env bash
# fp32 native kernels + NQ path + ATen-free step: targeted tests, fp32 bench/profile, bf16 bench/profile.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r6_b
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_f32_ops_gpu.py tests/test_fp32_gpu.py tests/test_kernels_gpu.py::test_sort_ids_is_a_stable_sort \
  tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_nq_gpu.py > "$O/pytest.log" 2>&1 || { tail -80 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 300 python bench.py --precision fp32 --batch 64 --steps 5 --warmup 2 > "$O/bench_fp32.log" 2>&1 || { tail -20 "$O/bench_fp32.log"; exit 1; }
tail -1 "$O/bench_fp32.log" | cut -c1-400
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
tools/gpu/step_prof.sh r6_b/step > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
python tools/kernel_table.py "$O/step/run_kernel_stats.csv" --steps 8 --top 80 > "$O/step/kernel_table.txt"
grep -iE "native|rocprim|sort_|key_bias|TOTAL" "$O/step/kernel_table.txt"
tools/gpu/step_prof.sh r6_b/step_fp32 --precision fp32 --batch 64 > /dev/null 2>&1 || { echo "fp32 profile failed"; exit 1; }
python tools/kernel_table.py "$O/step_fp32/run_kernel_stats.csv" --steps 8 --top 60 > "$O/step_fp32/kernel_table.txt"
head -40 "$O/step_fp32/kernel_table.txt"
