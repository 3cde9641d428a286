#!/usr/bin/env python
"""Persistent GEMM (v3) under CU contention: static vs dynamic (ticket) tile schedule.

On an 8-GPU node the RCCL all-reduce of a finished gradient bucket runs on the comm stream while the
backward's GEMMs run on the compute stream.  A GEMM workgroup needs a whole CU (142 KiB LDS, 512
threads at 2 waves/SIMD), so every CU an RCCL block holds delays one persistent workgroup — with a
static schedule that workgroup's whole 1/grid share of the tiles runs late.  This bench stands in for
the collective with ``cu_hog`` (``blocks`` workgroups, one per CU, spinning ``usec`` µs on a second
stream, launched just before the GEMM) and times the GEMM on its own stream, interleaved rounds in
one process, median of the rounds.

  python tools/gemm_contention_bench.py [--rounds 15] [--hogs 0,16,32,64] [--usec 200]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402
from tools.diag import cu_hog  # noqa: E402

SHAPES = (  # name, N, K, epi  (M = 98304 tokens: BERT-base, batch 256 x 384)
    ("ffn1_fwd_gelud", 3072, 768, 5),
    ("ffn2_dgrad_dmul", 3072, 768, 6),
    ("qkv_dgrad_resid", 768, 2304, 4),
    ("qkv_fwd_bias", 2304, 768, 1),
)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=98304)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--hogs", default="0,16,32,64")
    ap.add_argument("--usec", type=int, default=200)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    hogs = [int(h) for h in a.hogs.split(",")]
    M = a.M
    for name, N, K, epi in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        bias = torch.rand(N, device=dev)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = {"out": C}
        if epi in (1, 5):
            kw["bias"] = bias
        if epi in (5, 6):
            kw["pre"] = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
        if epi == 6:
            kw["part"] = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=dev)
        if epi == 4:
            kw["resid"] = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
        ref = None
        res = {}
        for sched in (0, 1):
            k.gemm_set_sched(sched)
            k.gemm_nt(A, B, epi, **kw)
            torch.cuda.synchronize()
            out = C.clone()
            if epi == 5:
                out = torch.cat([out, kw["pre"].clone()], 1)
            if ref is None:
                ref = out
            else:   # the schedule changes which CU computes a tile, never its value
                assert torch.equal(ref, out), f"{name}: dynamic schedule output differs from static"
        for _ in range(a.rounds):
            for sched in (0, 1):
                k.gemm_set_sched(sched)
                for h in hogs:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    if h:
                        with torch.cuda.stream(side):
                            cu_hog(h, a.usec)
                    e0.record(main_s)
                    k.gemm_nt(A, B, epi, **kw)
                    e1.record(main_s)
                    torch.cuda.synchronize()
                    res.setdefault((sched, h), []).append(e0.elapsed_time(e1) * 1e3)
        k.gemm_set_sched(0)
        fl = 2.0 * M * N * K
        for h in hogs:
            s0 = statistics.median(res[(0, h)])
            s1 = statistics.median(res[(1, h)])
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "hog_cus": h, "hog_us": a.usec if h else 0,
                              "static_us": round(s0, 1), "dynamic_us": round(s1, 1),
                              "static_tflops": round(fl / s0 / 1e6, 1), "dynamic_tflops": round(fl / s1 / 1e6, 1),
                              "dynamic_speedup": round(s0 / s1, 3)}), flush=True)


if __name__ == "__main__":
    main()
