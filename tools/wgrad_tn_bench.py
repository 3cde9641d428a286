#!/usr/bin/env python
"""dW = dyᵀ·x (fp32 out) at BERT shapes: hand-written TN split-K kernel (gemm_tn.hip) vs the
hipBLASLt batched split-K path, interleaved rounds in one process (median µs, TFLOP/s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402
from ml_recipe_distributed_pytorch_amd.ops import _wgrad_splits  # noqa: E402
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
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]
    for T in (24576, 98304):
        for N, K in shapes:
            dy = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
            x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
            g = torch.zeros(N, K, device=dev)
            s_auto = k.gemm_tn_splits(T, N, K)
            sb = _wgrad_splits(T, N, K)

            def blas():
                part = torch.bmm(dy.view(sb, T // sb, N).transpose(1, 2), x.view(sb, T // sb, K), out_dtype=torch.float32)
                torch.sum(part, 0, out=g)

            variants = {"blas": blas, "tn": lambda: k.gemm_tn(dy, x, g, False)}
            for s in sorted({max(1, s_auto // 2), s_auto * 2}):
                if T // 64 // s >= 2:
                    variants[f"tn_s{s}"] = (lambda s=s: k.gemm_tn(dy, x, g, False, s))
            k.gemm_tn(dy, x, g, False)
            ref = dy.float().t() @ x.float()
            err = ((g - ref).abs().max() / ref.abs().max()).item()
            times = {n: [] for n in variants}
            for _ in range(5):
                for n, f in variants.items():
                    times[n].append(timeit(f))
            fl = 2.0 * T * N * K
            row = {"T": T, "N": N, "K": K, "S": s_auto, "blas_splits": sb, "rel_err": round(err, 6)}
            for n, v in times.items():
                v.sort()
                row[n + "_us"] = round(v[2], 1)
                row[n + "_tf"] = round(fl / v[2] / 1e6, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
