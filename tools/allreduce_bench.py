#!/usr/bin/env python
"""All-reduce bandwidth of the native RCCL reducer (csrc/runtime/reducer.cpp) per message size — the
bucket-size side of the DDP replacement.  One process per GPU:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port 29511 \\
        tools/allreduce_bench.py [--sizes_mb 1,4,16,32,64,128,256] [--iters 20] [--dtype fp32|bf16]

(also runs as a single process: a 1-rank communicator).  Prints one JSON line per size with the time per
all-reduce, algorithm bandwidth (bytes / time) and ring bus bandwidth (algbw · 2(n-1)/n, the per-link
figure to compare against the ≈153 GB/s of one xGMI link × the links a ring uses).  NCCL_MIN_NCHANNELS /
NCCL_MAX_NCHANNELS in the environment select the RCCL channel count (bench.py --rccl_channels sets them).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes_mb", default="1,4,16,32,64,128,256")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    import torch.distributed as dist
    from ml_recipe_distributed_pytorch_amd.parallel import dist as hqdist
    from ml_recipe_distributed_pytorch_amd._native import kernels
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        info = hqdist.init_distributed("nccl")
        rank, dev = info.rank, info.device
    else:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        rank = 0
    k = kernels()
    uid = [bytes(k.rccl_unique_id()) if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    red = k.Reducer(rank, world, uid[0], dev.index)
    stream = torch.cuda.current_stream()
    for mb in (float(s) for s in a.sizes_mb.split(",")):
        n = int(mb * (1 << 20)) // 4
        buf = torch.ones(n, device=dev)
        scratch = torch.empty(n, dtype=torch.bfloat16, device=dev) if a.dtype == "bf16" else None

        def once():
            if scratch is None:
                red.allreduce_f32(buf.data_ptr(), n, stream.cuda_stream)
            else:
                red.allreduce_bf16(buf.data_ptr(), scratch.data_ptr(), n, stream.cuda_stream)
            red.wait(stream.cuda_stream)
        for _ in range(a.warmup):
            once()
        dist.barrier()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            once()
        ev[1].record()
        ev[1].synchronize()
        us = ev[0].elapsed_time(ev[1]) / a.iters * 1e3
        t = torch.tensor([us], device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        us = t.item()
        nbytes = n * (2 if scratch is not None else 4)
        algbw = nbytes / us / 1e3   # GB/s
        busbw = algbw * 2 * (world - 1) / world if world > 1 else 0.0
        if rank == 0:
            print(json.dumps({"world": world, "dtype": a.dtype, "size_mb": mb, "us": round(us, 1),
                              "algbw_GBs": round(algbw, 1), "busbw_GBs": round(busbw, 1),
                              "channels": os.environ.get("NCCL_MAX_NCHANNELS", "default")}), flush=True)
        del buf, scratch
    red.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
