#!/usr/bin/env python
"""Persistent NT GEMM (v3) at the b256 FFN1 / FFN2-dgrad / QKV / out-projection shapes: tile schedule (static /
dynamic per-XCD tickets) x start stagger of workgroup groups (gemm_set_stagger bits 0-7 = s_sleep(127) units,
bit 17 = four groups 0..3 x stagger instead of two), the half-tile tail kept on (bit 16).  The epilogue's stores
are a chip-wide burst when every CU reaches its tile seam at once (profiles/r5_epi_diag); desynchronising the
CUs spreads them under other CUs' mainloops.  Interleaved rounds in one process, median µs per config.

    python tools/gemm_stagger2.py [--T 98304] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

EPI = {"none": 0, "bias": 1, "resid": 4, "gelud": 5, "dmul": 6}
HALF, QUARTER = 1 << 16, 1 << 17


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=98304)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T = a.T
    configs = [("static", 0, 0), ("dyn", 0, 0), ("static", 1, 0), ("dyn", 1, 0), ("dyn", 2, 0),
               ("dyn", 1, QUARTER), ("dyn", 2, QUARTER), ("static", 1, QUARTER)]
    shapes = [(3072, 768, "gelud"), (3072, 768, "dmul"), (3072, 768, "none"), (2304, 768, "bias"),
              (768, 768, "bias")]
    for N, K, name in shapes:
        e = EPI[name]
        A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 0.2 - 0.1).bfloat16()
        kw = {"out": torch.empty(T, N, device=dev, dtype=torch.bfloat16)}
        if e in (1, 5):
            kw["bias"] = torch.rand(N, device=dev)
        if e in (5, 6):
            kw["pre"] = torch.randn(T, N, device=dev).bfloat16()
        if e == 6:
            kw["part"] = torch.empty(k.gemm_nt_part_rows(T, N, K), N, device=dev)
        res = {c: [] for c in configs}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(a.rounds):
            for c in configs:
                sched, stg, mode = c
                k.gemm_set_sched(1 if sched == "dyn" else 0)
                k.gemm_set_stagger(HALF | mode | stg)
                k.gemm_nt(A, B, e, **kw)
                ev[0].record()
                for _ in range(a.iters):
                    k.gemm_nt(A, B, e, **kw)
                ev[1].record()
                ev[1].synchronize()
                res[c].append(ev[0].elapsed_time(ev[1]) / a.iters * 1e3)
        k.gemm_set_sched(0)
        k.gemm_set_stagger(HALF)
        for c in configs:
            v = sorted(res[c])
            print(json.dumps({"N": N, "K": K, "epi": name, "sched": c[0], "stagger": c[1],
                              "groups": 4 if c[2] else 2, "us": round(v[len(v) // 2], 1)}), flush=True)


if __name__ == "__main__":
    main()
