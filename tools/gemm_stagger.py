#!/usr/bin/env python
"""Persistent NT GEMM (v3) at the b256 projection shapes vs its launch knobs (``gemm_set_stagger``): the
start offset of half of each XCD's workgroups (bits 0-7, units of s_sleep(127) ≈ 8128 cycles) and the
epilogue flags (bits 8-15: 1 nontemporal P stores, 2 nontemporal C stores, 4 no GELU math, 8 no stores —
the last two are diagnostics).  Interleaved rounds in one process; prints the median per (shape, knob).

    python tools/gemm_stagger.py [--T 98304] [--knobs 0,1,2,4] [--rounds 3]     # knob = stagger | flags << 8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

EPI = {"none": 0, "bias": 1, "resid": 4, "gelud": 5, "dmul": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=98304)
    ap.add_argument("--knobs", default="0,1,2,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T = a.T
    stg = [int(s, 0) for s in a.knobs.split(",")]
    shapes = [(3072, 768, "gelud"), (3072, 768, "dmul"), (3072, 768, "bias"), (768, 768, "resid"),
              (2304, 768, "bias"), (768, 2304, "resid")]
    if os.environ.get("KNOB_SHAPES"):
        keep = set(os.environ["KNOB_SHAPES"].split(","))
        shapes = [sh for sh in shapes if sh[2] in keep]
    k.gemm_set_variant(3)
    for N, K, name in shapes:
        e = EPI[name]
        A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 0.2 - 0.1).bfloat16()
        bias = torch.rand(N, device=dev)
        P = torch.randn(T, N, device=dev).bfloat16()
        R = torch.randn(T, N, device=dev).bfloat16()
        part = torch.empty(k.gemm_nt_part_rows(T, N, K), N, device=dev)
        kw = {}
        if e in (1, 5):
            kw["bias"] = bias
        if e in (5, 6):
            kw["pre"] = P
        if e == 6:
            kw["part"] = part
        if e == 4:
            kw["resid"] = R
        out = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        kw["out"] = out
        res = {s: [] for s in stg}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for s in stg:
                k.gemm_set_stagger(s | (1 << 16))
                k.gemm_nt(A, B, e, **kw)
                ev[0].record()
                for _ in range(a.iters):
                    k.gemm_nt(A, B, e, **kw)
                ev[1].record()
                ev[1].synchronize()
                res[s].append(ev[0].elapsed_time(ev[1]) / a.iters * 1e3)
        fl = 2.0 * T * N * K
        row = {"N": N, "K": K, "epi": name}
        for s in stg:
            us = sorted(res[s])[len(res[s]) // 2]
            row[f"k{s:#x}_us"] = round(us, 1)
        best = min(stg, key=lambda s: row[f"k{s:#x}_us"])
        row["best"] = hex(best)
        row["best_tflops"] = round(fl / row[f"k{best:#x}_us"] / 1e6, 1)
        print(json.dumps(row), flush=True)
        del A, B, P, R, part, out
    k.gemm_set_stagger(1 << 16)   # production word: half-tile tail on
    k.gemm_set_variant(0)


if __name__ == "__main__":
    main()
