#!/usr/bin/env bash
# GEMM schedule + reducer GPU tests, forced-reducer bench, and the 2-rank gloo rehearsal on one GPU (both
# ranks share cuda:0 and contend for its CUs: the dynamic v3 schedule's multi-process case).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-dp_sched}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gemm_sched_gpu.py tests/test_reducer_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python bench.py --force_reducer > "$O/bench_force_reducer.log" 2>&1 && tail -1 "$O/bench_force_reducer.log" | cut -c80-600 || { tail -20 "$O/bench_force_reducer.log"; exit 1; }
HQ_BENCH_BACKEND=gloo HQ_HANG_DUMP_S=120 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 --batch 32 > "$O/gloo2.log" 2>&1 && grep '"metric"' "$O/gloo2.log" | cut -c80-700 || { tail -30 "$O/gloo2.log"; exit 1; }
