"""Time the flash-attention kernels (ring forward, two-kernel backward) at BERT shapes, with and without
dropout; several interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).

Usage: python tools/attn_bench.py [--B 256] [--L 384] [--nh 12] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("HQ_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd._native import kernels  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--L", type=int, default=384)
    ap.add_argument("--nh", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    k = kernels()
    dev = torch.device("cuda")
    B, L, nh = a.B, a.L, a.nh
    H = nh * 64
    torch.manual_seed(0)
    qkv = torch.randn(B * L, 3 * H, device=dev, dtype=torch.bfloat16)
    kb = torch.zeros(B, L, device=dev)
    dctx = torch.randn(B * L, H, device=dev, dtype=torch.bfloat16)
    fl_fwd = 4.0 * B * nh * L * L * 64
    for rnd in range(a.rounds):
        for p in (0.0, 0.1):
            ctx, lse, bits = k.attn_fwd(qkv, kb, B, L, nh, p, 1, 1, 0.125)
            tf = timeit(lambda: k.attn_fwd(qkv, kb, B, L, nh, p, 1, 1, 0.125))
            tb = timeit(lambda: k.attn_bwd(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, True))
            print(f"round {rnd} p={p}: fwd {tf:8.1f} us ({fl_fwd / tf / 1e6:6.1f} TF)  "
                  f"bwd {tb:8.1f} us ({2.5 * fl_fwd / tb / 1e6:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
