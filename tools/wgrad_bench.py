#!/usr/bin/env python
"""dW = dyᵀ·x (fp32 out) at BERT shapes: split-K factor sweep for the batched-bmm formulation vs plain mm."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    dev = torch.device("cuda")
    for T in (24576, 98304):
        for N, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
            dy = torch.randn(T, N, device=dev).bfloat16()
            x = torch.randn(T, K, device=dev).bfloat16()
            g = torch.zeros(N, K, device=dev)
            row = {"T": T, "N": N, "K": K, "auto_s": _wgrad_splits(T, N, K)}
            fl = 2.0 * T * N * K
            row["mm_us"] = round(timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=g)), 1)
            for s in (2, 4, 8, 16, 32):
                if T % s:
                    continue
                def f(s=s):
                    part = torch.bmm(dy.view(s, T // s, N).transpose(1, 2), x.view(s, T // s, K), out_dtype=torch.float32)
                    torch.sum(part, 0, out=g)
                row[f"s{s}_us"] = round(timeit(f), 1)
            best = min((v, k) for k, v in row.items() if k.endswith("_us"))
            row["best"] = best[1]
            row["best_tflops"] = round(fl / best[0] / 1e6, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
