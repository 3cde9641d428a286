#!/usr/bin/env python
"""In-process interleaved A/B of the v3 NT GEMM's half-tile tail (flag word bit 16 of gemm_set_stagger) on the
BERT-base b256 step shapes whose tile count leaves a partial last wave, with a numerics check of every arm
against an fp32 torch product (epilogue applied in fp32).  K = 3072 shapes also run production v2
(gemm_set_variant(2)) so the v3 + half-tail arm can replace it where it wins.
Usage: tools/gemm_halftail_ab.py [reps] [M]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

HT = 1 << 16
# name, N, K, epi (0 none, 1 bias, 4 resid)
SHAPES = (("out_fwd_bias", 768, 768, 1), ("out_dgrad", 768, 768, 0), ("qkv_dgrad_resid", 768, 2304, 4),
          ("ffn2_fwd_bias_k3072", 768, 3072, 1), ("ffn1_dgrad_resid_k3072", 768, 3072, 4),
          ("qkv_fwd_bias", 2304, 768, 1))


def oracle(A, B, epi, kw, rows):
    y = A[rows].float() @ B.float().t()
    if epi == 1:
        y = y + kw["bias"]
    if epi == 4:
        y = y + kw["resid"][rows].float()
    return y


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 98304
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for name, N, K, epi in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        kw = {"out": torch.empty(M, N, device=dev, dtype=torch.bfloat16)}
        if epi == 1:
            kw["bias"] = torch.rand(N, device=dev)
        if epi == 4:
            kw["resid"] = torch.randn(M, N, device=dev).bfloat16()
        arms = [("v3", 3, 0), ("v3+halftail", 3, HT)]
        if K > 2304:
            arms = [("v2", 2, 0), ("v2+halftail", 2, HT)] + arms
        # rows checked: the first 2048 and the last 4096 (the half tiles live in the last wave)
        rows = torch.cat([torch.arange(0, 2048), torch.arange(M - 4096, M)]).to(dev)
        ref = oracle(A, B, epi, kw, rows)
        err = {}
        for an, var, w in arms:
            k.gemm_set_variant(var)
            k.gemm_set_stagger(w)
            kw["out"].fill_(float("nan"))
            k.gemm_nt(A, B, epi, **kw)
            torch.cuda.synchronize()
            o = kw["out"].float()
            err[an] = ((o[rows] - ref).abs().max() / ref.abs().max()).item()
            assert not torch.isnan(o).any(), (name, an, "unwritten outputs")
        res = {}
        for _ in range(reps):
            for an, var, w in arms:
                k.gemm_set_variant(var)
                k.gemm_set_stagger(w)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                k.gemm_nt(A, B, epi, **kw)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(an, []).append(e0.elapsed_time(e1) * 1e3)
        k.gemm_set_stagger(HT)
        k.gemm_set_variant(0)
        fl = 2.0 * M * N * K
        out = {"gemm": name}
        for an, _, _ in arms:
            t = statistics.median(res[an])
            out[an] = {"us": round(t, 1), "pf": round(fl / t / 1e9, 3), "relerr": float(f"{err[an]:.2e}")}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
