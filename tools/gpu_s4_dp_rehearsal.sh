#!/usr/bin/env bash
# Rehearse bench.py's multi-rank path (torchrun, reducer bucket hooks, barrier + MAX-reduced timing, rank-0 JSON)
# with 2 ranks sharing the one GPU of the box over gloo.  Throughput here means nothing; correctness of the path does.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s4_dp
mkdir -p $O
HQ_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --batch 32 > $O/dp2_gloo.log 2>&1 || { tail -40 $O/dp2_gloo.log; exit 1; }
grep -v amdgpu $O/dp2_gloo.log | tail -5
