#!/usr/bin/env python
"""The encoder GEMM shapes of small / irregular batches: own kernels (auto pick, forced 128² tiles, forced
256-row tiles where M % 256 == 0) vs hipBLASLt (torch.mm / addmm), interleaved rounds in one process.

    python tools/gemm_small_bench.py [--T 24576,1024,1268] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

SHAPES = [(2304, 768, "bias"), (768, 768, "bias"), (3072, 768, "bias"), (768, 3072, "bias"), (768, 768, "none"),
          (768, 2304, "none"), (3072, 768, "none")]
if os.environ.get("SMALL_SHAPES") == "epi":   # epilogue-heavy FFN shapes: own kernels only (no vendor twin)
    SHAPES = [(3072, 768, "gelud"), (3072, 768, "dmul"), (3072, 768, "bias"), (768, 768, "resid")]
EPI = {"none": 0, "bias": 1, "resid": 4, "gelud": 5, "dmul": 6}


def timeit(fn, iters):
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
    ap.add_argument("--T", default="24576,1024,1268")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    for T in (int(t) for t in a.T.split(",")):
        iters = 20 if T >= 8192 else 100
        for N, K, name in SHAPES:
            A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
            W = (torch.rand(N, K, device=dev) * 0.2 - 0.1).bfloat16()
            b = torch.rand(N, device=dev)
            bb = b.bfloat16()
            e = EPI[name]
            kw = {"bias": b} if e in (1, 5) else {}
            if e in (5, 6):
                kw["pre"] = torch.randn(T, N, device=dev).bfloat16()
            if e == 6:
                kw["part"] = None   # sized per kernel below
            if e == 4:
                kw["resid"] = torch.randn(T, N, device=dev).bfloat16()
            arms = {"auto": 0, "vS": 4}
            if T % 256 == 0:
                arms["v256"] = 3
            res = {n: [] for n in list(arms) + ["blas"]}
            for _ in range(a.rounds):
                for n, v in arms.items():
                    k.gemm_set_variant(v)
                    if e == 6:
                        kw["part"] = torch.empty(k.gemm_nt_part_rows(T, N, K), N, device=dev)
                    res[n].append(timeit(lambda: k.gemm_nt(A, W, e, **kw), iters))
                k.gemm_set_variant(0)
                if e == 1:
                    res["blas"].append(timeit(lambda: torch.addmm(bb, A, W.t()), iters))
                elif e == 0:
                    res["blas"].append(timeit(lambda: torch.mm(A, W.t()), iters))
                else:
                    res["blas"].append(float("nan"))
            k.gemm_set_variant(0)
            fl = 2.0 * T * N * K
            row = {"T": T, "N": N, "K": K, "epi": name, "pick": k.gemm_nt_supported(T, N, K)}
            for n, v in res.items():
                us = sorted(v)[len(v) // 2]
                row[n + "_us"] = round(us, 1)
            row["auto_tflops"] = round(fl / row["auto_us"] / 1e6, 1)
            row["auto_vs_blas"] = round(row["blas_us"] / row["auto_us"], 3)
            print(json.dumps(row), flush=True)
            del A, W


if __name__ == "__main__":
    main()
