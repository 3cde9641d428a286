#!/usr/bin/env bash
# Gradient-bucket / RCCL-channel sweep of the data-parallel training step, for an N-GPU node:
#   tools/gpu/bucket_sweep.sh <ngpus> [buckets_mb="8 16 32 64 128"] [channels="0 8 16 32"]
# Each point is `bench.py --gpus N --bucket_cap_mb B --rccl_channels C` under torch.distributed.run (one
# rank per GPU over RCCL; channels 0 = RCCL's default); with N = 1 the native reducer is forced active
# (--force_reducer), which exercises the whole bucket/all-reduce path on one GPU.  Prints one line per
# point: samples/s, ms/step, buckets, exposed comm wait and the comm span inside the backward.
# Also runs tools/allreduce_bench.py once per channel setting (message-size bandwidth curve).
set -o pipefail
cd "$(dirname "$0")/../.."
N=${1:-8}
BUCKETS=${2:-"8 16 32 64 128"}
CHANNELS=${3:-"0 8 16 32"}
O=gpurun_out/bucket_sweep_n$N
mkdir -p "$O"
port=29600
for c in $CHANNELS; do
  port=$((port + 1))
  envc=""
  [ "$c" != "0" ] && envc="NCCL_MIN_NCHANNELS=$c NCCL_MAX_NCHANNELS=$c"
  env $envc timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $port tools/allreduce_bench.py > "$O/allreduce_c$c.log" 2>&1 || { tail -20 "$O/allreduce_c$c.log"; exit 1; }
  grep '"size_mb"' "$O/allreduce_c$c.log"
  for b in $BUCKETS; do
    port=$((port + 1))
    extra=""
    [ "$N" = "1" ] && extra="--force_reducer"
    timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus "$N" --steps 20 --warmup 5 --bucket_cap_mb "$b" --rccl_channels "$c" $extra \
        > "$O/bench_b${b}_c$c.log" 2>&1 || { tail -20 "$O/bench_b${b}_c$c.log"; exit 1; }
    grep '"metric"' "$O/bench_b${b}_c$c.log" | python3 -c '
import json, sys
d = json.loads(sys.stdin.read())
print("bucket_mb=%s channels=%s samples_per_s=%.1f ms_per_step=%.2f buckets=%s comm_wait_ms=%s comm_span_ms=%s reducer=%s" % (
    "'"$b"'", "'"$c"'", d["value"], d["ms_per_step"], d.get("reducer_buckets"), d.get("comm_wait_ms"),
    d.get("comm_span_ms"), d.get("reducer")))' | tee -a "$O/summary.txt"
  done
done
