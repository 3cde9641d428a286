#!/bin/bash
# Round-3 check: GPU suite, headline bench, and the reference's literal workload (train_batch_size 256 as
# 128 micro-batches of 2 at seq 512) eager vs HIP-graph replay, with the forced native-RCCL reducer.
set -o pipefail
O=gpurun_out/${1:-r3g}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_headline.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --batch 256 --batch_split 128 --seq 512 --steps 3 --warmup 1 > $O/bench_ref_eager.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --batch 256 --batch_split 128 --seq 512 --steps 3 --warmup 1 --graph > $O/bench_ref_graph.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 1 --batch 256 --batch_split 128 --seq 512 --steps 3 --warmup 1 --graph --force_reducer > $O/bench_ref_graph_reducer.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --batch 256 --seq 512 --steps 10 --warmup 3 > $O/bench_merged_s512.log 2>&1 || exit 1
