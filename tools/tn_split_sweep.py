#!/usr/bin/env python
"""Weight-gradient TN GEMM: time per split count S on the BERT-base b256 wgrad shapes (median of N
interleaved launches).  Usage: tools/tn_split_sweep.py [reps]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

SHAPES = (("qkv", 2304, 768, (4, 6, 8, 9, 12, 18)), ("out", 768, 768, (14, 16, 20, 24, 28, 32, 56)),
          ("ffn1", 3072, 768, (4, 6, 7, 8, 10, 14)), ("ffn2", 768, 3072, (4, 6, 7, 8, 10, 14)))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    T = 98304
    for name, N, K, splits in SHAPES:
        dy = (torch.randn(T, N, device=dev) * 0.1).bfloat16()
        x = torch.randn(T, K, device=dev).bfloat16()
        out = torch.empty(N, K, device=dev)
        ref = None
        res = {S: [] for S in splits}
        for _ in range(reps):
            for S in splits:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                k.gemm_tn(dy, x, out, False, S)
                e1.record()
                torch.cuda.synchronize()
                res[S].append(e0.elapsed_time(e1) * 1e3)
                if ref is None:
                    ref = out.clone()
                else:
                    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-3), (name, S)
        fl = 2.0 * T * N * K
        print(json.dumps({"wgrad": name, "auto_S": k.gemm_tn_splits(T, N, K),
                          **{f"S{S}": [round(statistics.median(v), 1), round(fl / statistics.median(v) / 1e9, 3)]
                             for S, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
