#!/usr/bin/env python
"""Epilogue cost of the MFMA NT GEMM at the b256 shapes: the same A·Bᵀ timed with each epilogue, so
time(EPI) - time(NONE) is what the fused elementwise work and its extra HBM traffic cost.

    python tools/gemm_epi_bench.py [--T 98304]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

EPI = {"none": 0, "bias": 1, "gelu": 2, "dgelu": 3, "resid": 4, "gelud": 5, "dmul": 6}


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
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    T = a.T
    for N, K, epis in ((3072, 768, ("none", "bias", "gelud", "dmul", "gelu", "dgelu")), (768, 768, ("none", "bias", "resid")),
                       (2304, 768, ("none", "bias")), (768, 3072, ("none", "bias")), (768, 2304, ("none", "resid"))):
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
            ts = sorted(timeit(fn) for _ in range(5))
            print(json.dumps({"T": T, "N": N, "K": K, "epi": name, "us": round(ts[2], 1),
                              "tflops": round(fl / ts[2] / 1e6, 1)}), flush=True)
        del A, B, P, R, part, C


if __name__ == "__main__":
    main()
