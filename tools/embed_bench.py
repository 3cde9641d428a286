#!/usr/bin/env python
"""embed_bwd cost split at the b256 shape: full kernel vs. position atomics disabled (every pos id =
pad_pos) vs. word atomics disabled (every id = pad_word)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd._native import kernels  # noqa: E402


def timeit(fn, iters=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    ev[1].synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1e3


def main():
    k = kernels()
    dev = torch.device("cuda")
    B, L, H, V, P = 256, 384, 768, 30522, 512
    T = B * L
    ids = torch.randint(1, V, (T,), device=dev)
    pids = torch.arange(L, device=dev).repeat(B)
    tids = (torch.arange(L, device=dev) > 66).long().repeat(B)
    ww = (torch.randn(V, H, device=dev) * 0.02).bfloat16()
    wp = (torch.randn(P, H, device=dev) * 0.02).bfloat16()
    wt = (torch.randn(2, H, device=dev) * 0.02).bfloat16()
    g, b = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    y, mean, rstd = k.embed_fwd(ids, pids, tids, ww, wp, wt, g, b, 1e-12, 0.1, 1, 0)
    dy = torch.randn(T, H, device=dev).bfloat16()
    gw, gp, gt = torch.zeros(V, H, device=dev), torch.zeros(P, H, device=dev), torch.zeros(2, H, device=dev)
    gg, gb = torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    for name, i, p, pw, pp in (("full", ids, pids, 0, -1), ("no_pos_atomics", ids, torch.full_like(pids, 511), 0, 511),
                              ("no_word_atomics", torch.zeros_like(ids), pids, 0, -1),
                              ("no_atomics", torch.zeros_like(ids), torch.full_like(pids, 511), 0, 511)):
        us = timeit(lambda: k.embed_bwd(dy, i, p, tids, ww, wp, wt, g, mean, rstd, 0.1, 1, 0, gw, gp, gt, gg, gb,
                                        False, pw, pp, L))
        print(f"embed_bwd {name:16s} {us:8.1f} us")
    print(f"embed_fwd {timeit(lambda: k.embed_fwd(ids, pids, tids, ww, wp, wt, g, b, 1e-12, 0.1, 1, 0)):8.1f} us")


if __name__ == "__main__":
    main()
