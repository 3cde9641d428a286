#!/usr/bin/env python
"""Tile order of the persistent NT GEMM: M-major rows (band 0) vs column bands of `band` tiles (flag word bits
18-21, gemm_set_stagger), interleaved per shape / epilogue at the b256 BERT shapes.

    python tools/gemm_band_bench.py [--T 98304] [--bands 0,6,4,3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

EPI = {"none": 0, "bias": 1, "gelu": 2, "dgelu": 3, "resid": 4, "gelud": 5, "dmul": 6}
HALF_TAIL = 1 << 16


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=98304)
    ap.add_argument("--bands", default="0,6,4,3,2,1")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    bands = [int(b) for b in a.bands.split(",")]
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    T = a.T
    for N, K, epis in ((3072, 768, ("bias", "gelud", "dmul")), (2304, 768, ("bias",)), (768, 768, ("bias", "resid")),
                       (768, 3072, ("bias", "none")), (768, 2304, ("resid",))):
        A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 0.2 - 0.1).bfloat16()
        bias = torch.rand(N, device=dev)
        P = torch.randn(T, N, device=dev).bfloat16()
        R = torch.randn(T, N, device=dev).bfloat16()
        part = torch.empty(k.gemm_nt_part_rows(T, N, K), N, device=dev)
        C = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        for name in epis:
            e = EPI[name]
            kw = {"out": C}
            if e in (1, 2, 5):
                kw["bias"] = bias
            if e in (2, 3, 5, 6):
                kw["pre"] = P
            if e in (3, 6):
                kw["part"] = part
            if e == 4:
                kw["resid"] = R
            fn = lambda: k.gemm_nt(A, B, e, **kw)  # noqa: E731
            bs = [b for b in bands if b == 0 or b < N // 256]
            ts = {b: [] for b in bs}
            ref = None
            for _ in range(a.reps):
                for b in bs:
                    k.gemm_set_stagger(HALF_TAIL | (b << 18))
                    ts[b].append(timeit(fn))
                    if ref is None:
                        ref = C.clone()
                    elif not torch.equal(ref, C):
                        raise SystemExit(f"band {b}: output differs from band 0 at N={N} K={K} {name}")
            k.gemm_set_stagger(HALF_TAIL)
            row = {b: round(sorted(v)[len(v) // 2], 1) for b, v in ts.items()}
            print(json.dumps({"N": N, "K": K, "epi": name, "us_by_band": row,
                              "best": min(row, key=row.get), "tflops0": round(fl / row[0] / 1e6, 1)}), flush=True)
        del A, B, P, R, part, C


if __name__ == "__main__":
    main()
