#!/usr/bin/env python
"""Our MFMA NT GEMM vs hipBLASLt (torch, TunableOp results loaded) on the BERT projection shapes.
Interleaved rounds in one process; median µs and TFLOP/s."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402
from ml_recipe_distributed_pytorch_amd.ops.tuning import enable_tuned_gemms  # noqa: E402


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
    enable_tuned_gemms()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    out = []
    for T in (24576, 98304):
        for name, N, K, epi in (("qkv_fwd", 2304, 768, 1), ("out_fwd", 768, 768, 1), ("ffn1_fwd", 3072, 768, 1),
                                ("ffn2_fwd", 768, 3072, 1), ("qkv_dgrad", 768, 2304, 0), ("ffn1_dgrad", 768, 3072, 0),
                                ("ffn2_dgrad", 3072, 768, 0)):
            A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
            B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
            bias = torch.rand(N, device=dev)
            C = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            Bt = B.t().contiguous()
            bias16 = bias.bfloat16()
            ours = (lambda: k.gemm_nt(A, B, epi, bias=bias, out=C)) if epi else (lambda: k.gemm_nt(A, B, 0, out=C))
            theirs = (lambda: torch.addmm(bias16, A, B.t(), out=C)) if epi else (lambda: torch.mm(A, Bt, out=C))
            ref = A.float() @ B.float().t() + (bias if epi else 0)
            ours()
            err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
            a, b, c = [], [], []
            for _ in range(5):
                a.append(timeit(ours))
                b.append(timeit(theirs))
                k.gemm_set_variant(1)
                c.append(timeit(ours))
                k.gemm_set_variant(0)
            a.sort(), b.sort(), c.sort()
            fl = 2.0 * T * N * K
            row = {"T": T, "gemm": name, "N": N, "K": K, "ours_us": round(a[2], 1), "v1_us": round(c[2], 1),
                   "hipblaslt_us": round(b[2], 1),
                   "ours_tflops": round(fl / a[2] / 1e6, 1), "v1_tflops": round(fl / c[2] / 1e6, 1),
                   "hipblaslt_tflops": round(fl / b[2] / 1e6, 1),
                   "speedup": round(b[2] / a[2], 3), "rel_err": round(err, 5)}
            print(json.dumps(row), flush=True)
            out.append(row)
        # fused epilogues vs hipBLASLt + the separate elementwise kernel
        for name, N, K in (("ffn1_fwd+gelu", 3072, 768), ("ffn2_dgrad+dgelu", 3072, 768)):
            A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
            B = (torch.rand(N, K, device=dev) * 0.2 - 0.1).bfloat16()
            bias = torch.rand(N, device=dev)
            pre = (torch.randn(T, N, device=dev)).bfloat16()
            gb = torch.zeros(N, device=dev)
            Bt = B.t().contiguous()
            part = torch.empty(k.gemm_nt_part_rows(T, N, K), N, device=dev)
            if "gelu" in name and "dgelu" not in name:
                P = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
                ours = lambda: k.gemm_nt(A, B, 2, bias=bias, pre=P)
                theirs = lambda: k.gelu_fwd(torch.addmm(bias.bfloat16(), A, B.t()))
            else:
                def ours():
                    d = k.gemm_nt(A, B, 3, pre=pre, part=part)
                    k.colsum_into(part, gb, False)
                    return d
                theirs = lambda: k.gelu_bwd(torch.mm(A, Bt), pre, gb, False)
            a, b, c = [], [], []
            for _ in range(5):
                a.append(timeit(ours))
                b.append(timeit(theirs))
                k.gemm_set_variant(1)
                c.append(timeit(ours))
                k.gemm_set_variant(0)
            a.sort(), b.sort(), c.sort()
            row = {"T": T, "gemm": name, "N": N, "K": K, "ours_us": round(a[2], 1), "v1_us": round(c[2], 1),
                   "hipblaslt+ew_us": round(b[2], 1),
                   "speedup": round(b[2] / a[2], 3)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
