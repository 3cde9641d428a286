#!/usr/bin/env python
"""Weight-gradient TN GEMM with and without the fused bias gradient, interleaved in one process (median of
N), on the BERT-base b256 wgrad shapes: the bias arm's overhead is the fused column-sum's cost.
Usage: tools/tn_bias_bench.py [reps]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

SHAPES = (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    T = 98304
    for name, N, K in SHAPES:
        dy = (torch.randn(T, N, device=dev) * 0.1).bfloat16()
        x = torch.randn(T, K, device=dev).bfloat16()
        out = torch.empty(N, K, device=dev)
        db = torch.empty(N, device=dev)
        k.gemm_tn(dy, x, out, False, 0, db)
        torch.cuda.synchronize()
        ref_db = dy.float().sum(0)
        db_err = ((db - ref_db).abs().max() / ref_db.abs().max()).item()
        res = {"plain": [], "bias": []}
        for _ in range(reps):
            for arm in ("plain", "bias"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if arm == "bias":
                    k.gemm_tn(dy, x, out, False, 0, db)
                else:
                    k.gemm_tn(dy, x, out, False)
                e1.record()
                torch.cuda.synchronize()
                res[arm].append(e0.elapsed_time(e1) * 1e3)
        p, b = statistics.median(res["plain"]), statistics.median(res["bias"])
        fl = 2.0 * T * N * K
        print(json.dumps({"wgrad": name, "N": N, "K": K, "splits": k.gemm_tn_splits(T, N, K), "plain_us": round(p, 1),
                          "bias_us": round(b, 1), "bias_overhead": round(b / p - 1, 3), "plain_pf": round(fl / p / 1e9, 3),
                          "db_relerr": float(f"{db_err:.2e}")}), flush=True)


if __name__ == "__main__":
    main()
