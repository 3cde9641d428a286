"""Time the flash-attention kernels (fwd, full bwd) at BERT shapes, with and without dropout, and A/B the
forward variants (HQ_ATTN_FWD=2: whole-head-resident v2, 3: LDS-DMA ring v3) in one process.

Usage: python tools/attn_bench.py [--B 256] [--L 384] [--nh 12] [--fwd 2,3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    ap.add_argument("--fwd", default="2,3:2,3:4", help="variants: HQ_ATTN_FWD[:HQ_ATTN_AHEAD], comma-separated")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--bwd", default="2,3", help="backward variants (HQ_ATTN_BWD), comma-separated")
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
    variants = [v for v in a.fwd.split(",") if v]
    for p in (0.0, 0.1):
        outs = {}
        for rnd in range(a.rounds):  # interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)
            for v in variants:
                os.environ["HQ_ATTN_FWD"] = v.split(":")[0]
                if ":" in v:
                    os.environ["HQ_ATTN_AHEAD"] = v.split(":")[1]
                ctx, lse, bits = k.attn_fwd(qkv, kb, B, L, nh, p, 1, 1, 0.125)
                outs[v] = (ctx, lse, bits)
                tf = timeit(lambda: k.attn_fwd(qkv, kb, B, L, nh, p, 1, 1, 0.125))
                print(f"p={p} fwd v{v} round {rnd}: {tf:8.1f} us ({fl_fwd / tf / 1e6:6.1f} TF)", flush=True)
        if len(variants) > 1:
            r = outs[variants[0]]
            for v in variants[1:]:
                o = outs[v]
                dc = (o[0].float() - r[0].float()).abs().max().item()
                dl = (o[1] - r[1]).abs().max().item()
                same_bits = p == 0 or torch.equal(o[2], r[2])
                print(f"p={p} v{v} vs v{variants[0]}: max|dctx| {dc:.3e} max|dlse| {dl:.3e} bits_equal {same_bits}")
        ctx, lse, bits = outs[variants[-1]]
        os.environ.pop("HQ_ATTN_AHEAD", None)
        grads = {}
        for rnd in range(a.rounds):
            for v in [x for x in a.bwd.split(",") if x]:
                os.environ["HQ_ATTN_BWD"] = v
                grads[v] = k.attn_bwd(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False)
                tb = timeit(lambda: k.attn_bwd(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False))
                print(f"p={p} bwd v{v} round {rnd}: {tb:8.1f} us ({2.5 * fl_fwd / tb / 1e6:6.1f} TF)", flush=True)
        vs = list(grads)
        for v in vs[1:]:
            d = (grads[v].float() - grads[vs[0]].float()).abs()
            H3 = grads[v].shape[1] // 3
            print(f"p={p} bwd v{v} vs v{vs[0]}: max|d dq| {d[:, :H3].max().item():.3e} "
                  f"max|d dk| {d[:, H3:2 * H3].max().item():.3e} max|d dv| {d[:, 2 * H3:].max().item():.3e}")
        os.environ.pop("HQ_ATTN_BWD", None)


if __name__ == "__main__":
    main()
