#!/usr/bin/env python
"""LayerNorm kernels at the b256 BERT-base shape (T = 98304, H = 768, dropout 0.1): fwd, bwd without and
with the second upstream gradient, and the effective HBM bandwidth of each.

    python tools/ln_bench.py [--T 98304] [--H 768]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd._native import kernels  # noqa: E402


def timeit(fn, iters=30):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    ev[1].synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=98304)
    ap.add_argument("--H", type=int, default=768)
    a = ap.parse_args()
    k = kernels()
    dev = torch.device("cuda")
    T, H = a.T, a.H
    x = torch.randn(T, H, device=dev).bfloat16()
    r = torch.randn(T, H, device=dev).bfloat16()
    g, b = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    _, z, mean, rstd = k.ln_fwd(x, r, g, b, 1e-12, 0.1, 1, 0)
    dy = torch.randn(T, H, device=dev).bfloat16()
    gg, gb, gbias = torch.zeros(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    mb = T * H * 2 / 1e6
    st8 = torch.zeros(4, device=dev)
    for name, fn, nbytes in (
            ("ln_fwd", lambda: k.ln_fwd(x, r, g, b, 1e-12, 0.1, 1, 0), 4 * mb),
            ("ln_fwd + e4m3 (fp8)", lambda: k.ln_fwd(x, r, g, b, 1e-12, 0.1, 1, 0, q8=st8, phase=0), 4.5 * mb),
            ("ln_bwd (dy)", lambda: k.ln_bwd(dy, None, z, g, mean, rstd, 0.1, 1, 0, gg, gb, gbias, False), 4 * mb),
            ("ln_bwd (dy + dy2)", lambda: k.ln_bwd(dy, r, z, g, mean, rstd, 0.1, 1, 0, gg, gb, gbias, False), 5 * mb)):
        us = sorted(timeit(fn) for _ in range(5))[2]
        print(f"{name:20s} {us:8.1f} us  {nbytes / us:6.2f} TB/s (row tensors only)")


if __name__ == "__main__":
    main()
