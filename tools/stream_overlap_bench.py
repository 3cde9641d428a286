"""Cost of cross-stream work beside a compute stream (diagnostic for the gradient reducer).

A compute stream runs a chain of GEMMs; every `every` GEMMs it records an event that a second stream
waits on before doing `side` work: none | tiny (a 1-element add) | copy (a 32 MiB device copy, what a
1-rank RCCL all-reduce amounts to) | rccl (the native reducer's all-reduce of a 32 MiB bucket, ncclAvg, high-priority comm stream)
| rccl_lo (normal-priority comm stream) | rccl_sum (ncclSum) | torchpg (torch.distributed all_reduce, SUM, on a side stream).
Reports ms per GEMM chain for each variant (interleaved rounds in one process).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    buf = torch.randn(8 << 20, device=dev)
    buf2 = torch.empty_like(buf)
    side = torch.cuda.Stream(priority=-1)
    red = None
    from ml_recipe_distributed_pytorch_amd._native import kernels
    k = kernels()
    os.environ["HQ_COMM_PRIO"] = "1"  # communicator whose comm stream has high priority
    red = k.Reducer(0, 1, bytes(k.rccl_unique_id()), 0)
    os.environ["HQ_COMM_PRIO"] = "0"  # ... and one at normal priority (the default)
    red_lo = k.Reducer(0, 1, bytes(k.rccl_unique_id()), 0)
    n = 48

    def chain(mode, every=4):
        cur = torch.cuda.current_stream()
        for i in range(n):
            torch.mm(a, b)
            if mode != "none" and i % every == every - 1:
                if mode == "rccl":
                    red.allreduce_f32(buf.data_ptr(), buf.numel(), cur.cuda_stream)
                    continue
                if mode == "rccl_nowait":
                    red.allreduce_f32(buf.data_ptr(), buf.numel(), cur.cuda_stream)
                    continue
                if mode == "rccl_lo":
                    red_lo.allreduce_f32(buf.data_ptr(), buf.numel(), cur.cuda_stream)
                    continue
                if mode == "rccl_sum":
                    red.allreduce_f32(buf.data_ptr(), buf.numel(), cur.cuda_stream, 1)
                    continue
                if mode == "torchpg":
                    import torch.distributed as dist
                    with torch.cuda.stream(side):
                        side.wait_stream(cur)
                        dist.all_reduce(buf)
                    continue
                ev = torch.cuda.Event()
                ev.record(cur)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    if mode == "tiny":
                        buf[:1].add_(1.0)
                    elif mode == "copy":
                        buf2.copy_(buf)
        if mode in ("rccl", "rccl_sum"):
            red.wait(cur.cuda_stream)
        elif mode == "rccl_lo":
            red_lo.wait(cur.cuda_stream)
        elif mode == "rccl_nowait":
            pass
        else:
            cur.wait_stream(side)

    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    modes = [m for m in os.environ.get("SOB_MODES", "none,rccl,none,rccl_lo,none,rccl_sum,none,torchpg").split(",")]
    for m in modes:
        chain(m)
    torch.cuda.synchronize()
    for rnd in range(2):
        for m in modes:
            torch.cuda.synchronize()
            t = time.perf_counter()
            chain(m)
            torch.cuda.synchronize()
            print(f"round {rnd} {m:12s}: {(time.perf_counter() - t) * 1e3:8.2f} ms / {n} GEMMs", flush=True)


if __name__ == "__main__":
    main()
