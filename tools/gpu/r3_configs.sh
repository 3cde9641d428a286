#!/usr/bin/env bash
# Every BASELINE config that runs on one GPU, on one box (round-3 final): bf16 headline, fp8 (config #5),
# BERT-large seq 512, the reference's 128 x 2 x 512 accumulation workload, and the torchrun world-1 path
# with the native RCCL reducer forced (the code path of the 8-GPU run).
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_configs}
mkdir -p "$O"
summ() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["unit"], d["ms_per_step"], "ms/step, mem", d.get("max_mem_gb"), "GB, reducer", d.get("reducer"), "world", d.get("world_size"))'; }
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; exit 1; }; echo "$name $(tail -1 "$O/$name.log" | summ)"; }
run bf16_b256 --steps 20
run fp8_b256 --precision fp8 --steps 20
run large512_b64 --model bert-large-uncased --seq 512 --batch 64 --steps 10 --warmup 3
run ref_workload_2x128_s512 --batch 256 --batch_split 128 --seq 512 --steps 2 --warmup 1
timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --force_reducer --steps 20 > "$O/torchrun_forced_reducer.log" 2>&1 || { tail -20 "$O/torchrun_forced_reducer.log"; exit 1; }
echo "torchrun_forced_reducer $(grep '^{' "$O/torchrun_forced_reducer.log" | tail -1 | summ)"
