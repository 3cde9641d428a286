#!/usr/bin/env python
"""In-process interleaved A/B of the v3 NT GEMM's two MFMA forms (16x16x32 vs 32x32x16, flag bit 16 of
gemm_set_stagger) on the BERT-base b256 step shapes, with a numerics check of each form's output against
an fp32 torch product (the epilogue math applied in fp32).  K = 3072 shapes are forced onto v3
(gemm_set_variant(3)) so both forms see every projection shape.
Usage: tools/gemm_mfma32_ab.py [reps]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

M32 = 1 << 16
# name, N, K, epi (0 none, 1 bias, 4 resid, 5 gelud, 6 dmul)
SHAPES = (("qkv_fwd_bias", 2304, 768, 1), ("out_fwd_bias", 768, 768, 1), ("ffn1_fwd_gelud", 3072, 768, 5),
          ("ffn2_dgrad_dmul", 3072, 768, 6), ("qkv_dgrad_resid", 768, 2304, 4), ("out_dgrad", 768, 768, 0),
          ("ffn2_fwd_bias_k3072", 768, 3072, 1), ("ffn1_dgrad_k3072", 768, 3072, 4))


def oracle(A, B, epi, kw):
    y = A.float() @ B.float().t()
    if epi in (1, 5):
        y = y + kw["bias"]
    if epi == 4:
        y = y + kw["resid"].float()
    if epi == 5:
        y = torch.nn.functional.gelu(y)
    if epi == 6:
        y = y * kw["pre"].float()
    return y


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    M = 98304
    torch.manual_seed(0)
    for name, N, K, epi in SHAPES:
        k.gemm_set_variant(3 if K > 2304 else 0)
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        kw = {"out": torch.empty(M, N, device=dev, dtype=torch.bfloat16)}
        if epi in (1, 5):
            kw["bias"] = torch.rand(N, device=dev)
        if epi in (5, 6):
            kw["pre"] = torch.rand(M, N, device=dev).bfloat16()
        if epi == 6:
            kw["part"] = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=dev)
        if epi == 4:
            kw["resid"] = torch.randn(M, N, device=dev).bfloat16()
        pre_in = kw["pre"].clone() if epi == 6 else None
        ref = oracle(A[:4096], B, epi, {**kw, "pre": pre_in[:4096]} if epi == 6 else kw)
        err = {}
        for w in (0, M32):
            k.gemm_set_stagger(w)
            k.gemm_nt(A, B, epi, **kw)
            torch.cuda.synchronize()
            err[w] = ((kw["out"][:4096].float() - ref).abs().max() / ref.abs().max()).item()
        res = {}
        for _ in range(reps):
            for w in (0, M32):
                k.gemm_set_stagger(w)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                k.gemm_nt(A, B, epi, **kw)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(w, []).append(e0.elapsed_time(e1) * 1e3)
        k.gemm_set_stagger(0)
        k.gemm_set_variant(0)
        t16, t32 = statistics.median(res[0]), statistics.median(res[M32])
        fl = 2.0 * M * N * K
        print(json.dumps({"gemm": name, "us_16x16x32": round(t16, 1), "us_32x32x16": round(t32, 1),
                          "pf_16": round(fl / t16 / 1e9, 3), "pf_32": round(fl / t32 / 1e9, 3),
                          "speedup": round(t16 / t32, 3), "relerr_16": float(f"{err[0]:.2e}"),
                          "relerr_32": float(f"{err[M32]:.2e}")}), flush=True)


if __name__ == "__main__":
    main()
