#!/usr/bin/env python
"""In-process interleaved A/B of persistent-GEMM (v3) flag words (gemm_set_stagger: bits 0-7 stagger in
units of s_sleep(127), bits 8-15 HQ_GEMM_EPIFLAGS diagnostics, bit 16 the half-tile tail — kept on in every
arm unless a word sets bit 17, which turns it off) on the BERT-base b256 shapes that run on v3.
Usage: tools/gemm_knob_ab.py 0 0x2 [...]  (default: 0 vs stagger 2)"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

SHAPES = (("qkv_fwd_bias", 2304, 768, 1), ("out_fwd_bdr", 768, 768, 7), ("ffn1_fwd_gelud", 3072, 768, 5),
          ("ffn2_dgrad_dmul", 3072, 768, 6), ("qkv_dgrad_resid", 768, 2304, 4), ("out_dgrad", 768, 768, 0))


def main():
    words = [int(w, 0) for w in sys.argv[1:]] or [0, 2]
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    M = 98304
    for name, N, K, epi in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        kw = {"out": torch.empty(M, N, device=dev, dtype=torch.bfloat16)}
        if epi in (1, 5, 7):
            kw["bias"] = torch.rand(N, device=dev)
        if epi in (5, 6):
            kw["pre"] = torch.rand(M, N, device=dev).bfloat16()
        if epi == 6:
            kw["part"] = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=dev)
        if epi in (4, 7):
            kw["resid"] = torch.randn(M, N, device=dev).bfloat16()
        if epi == 7:
            kw.update(p=0.1, seed=1, opid=2)
        res = {}
        for _ in range(11):
            for w in words:
                k.gemm_set_stagger((w & 0xFFFF) | (0 if w & (1 << 17) else 1 << 16))
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                k.gemm_nt(A, B, epi, **kw)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(w, []).append(e0.elapsed_time(e1) * 1e3)
        k.gemm_set_stagger(1 << 16)
        print(json.dumps({"gemm": name, **{hex(w): round(statistics.median(v), 1) for w, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
