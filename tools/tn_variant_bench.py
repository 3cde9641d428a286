#!/usr/bin/env python
"""Weight-gradient TN GEMM: the alternating-row kernel (variant 5) vs the lockstep kernel (variant 1) on the
BERT-base b256 wgrad shapes, median of interleaved launches (split-K reduce included), outputs compared bitwise.

    python tools/tn_variant_bench.py [reps]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

SHAPES = (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    T = 98304
    for name, N, K in SHAPES:
        dy = (torch.randn(T, N, device=dev) * 0.1).bfloat16()
        x = torch.randn(T, K, device=dev).bfloat16()
        vs = [int(v) for v in os.environ.get("TN_VARIANTS", "5,1").split(",")]
        outs = {v: torch.empty(N, K, device=dev) for v in vs}
        res = {v: [] for v in vs}
        for _ in range(reps):
            for v in vs:
                k.gemm_tn_set_variant(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                k.gemm_tn(dy, x, outs[v], False)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1e3)
        k.gemm_tn_set_variant(0)
        fl = 2.0 * T * N * K
        med = {v: statistics.median(res[v]) for v in vs}
        print(json.dumps({"wgrad": name, "S": k.gemm_tn_splits(T, N, K),
                          **{f"us_v{v}": round(med[v], 1) for v in vs}, **{f"pf_v{v}": round(fl / med[v] / 1e9, 3) for v in vs},
                          "bitwise_v1": bool(torch.equal(outs[vs[0]], outs[1])) if 1 in vs else None}), flush=True)


if __name__ == "__main__":
    main()
