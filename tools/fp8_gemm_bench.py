#!/usr/bin/env python
"""Forward-projection GEMMs at b256: own fp8 kernel (gemm_fp8.hip) vs hipBLASLt fp8 (torch._scaled_mm)
vs own bf16 v2 kernel; interleaved rounds in one process, median µs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402
from ml_recipe_distributed_pytorch_amd.ops.tuning import enable_tuned_gemms  # noqa: E402


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    enable_tuned_gemms()
    k = _native.kernels()
    dev = torch.device("cuda")
    T = 98304
    for name, N, K in (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
        A = torch.randn(T, K, device=dev).bfloat16()
        B = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        A8, sa = k.fp8_quantize(A)
        B8, sb = k.fp8_quantize(B)
        sa, sb = sa.reshape(1).float(), sb.reshape(1).float()
        ours = lambda: k.gemm_fp8(A8, B8, 1, bias, sa, sb)
        blas = lambda: torch._scaled_mm(A8, B8.t(), scale_a=sa.reshape(()), scale_b=sb.reshape(()), bias=bias.bfloat16(),
                                        out_dtype=torch.bfloat16)
        bf16 = lambda: k.gemm_nt(A, B, 1, bias=bias)
        t = {"fp8_own": [], "fp8_hipblaslt": [], "bf16_own": []}
        for _ in range(5):
            t["fp8_own"].append(timeit(ours))
            t["fp8_hipblaslt"].append(timeit(blas))
            t["bf16_own"].append(timeit(bf16))
        fl = 2.0 * T * N * K
        row = {"gemm": name, "T": T, "N": N, "K": K}
        for kk, v in t.items():
            v.sort()
            row[kk + "_us"] = round(v[2], 1)
            row[kk + "_tf"] = round(fl / v[2] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
