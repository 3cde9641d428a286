"""fp8 GEMM: per-tile v2 vs persistent form on the BERT-base b256 step shapes (M = 98304 tokens), interleaved
rounds in one process, median µs per call.  Usage: python tools/fp8_lab/fp8_variant_bench.py [--rounds 7]"""
import argparse
import sys
import os

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

EPI_NONE, EPI_BIAS, EPI_RESID, EPI_GELUD, EPI_DMUL = 0, 1, 4, 5, 6
SHAPES = [  # name, N, K, epi, q8, write_out
    ("qkv_fwd+bias", 2304, 768, EPI_BIAS, False, True),
    ("out_fwd+bias", 768, 768, EPI_BIAS, False, True),
    ("ffn2_fwd+bias", 768, 3072, EPI_BIAS, False, True),
    ("ffn1_fwd+gelu'+e4m3", 3072, 768, EPI_GELUD, True, False),
    ("ffn2_dgrad*gelu'+e5m2", 3072, 768, EPI_DMUL, True, False),
    ("ffn1_dgrad", 768, 3072, EPI_NONE, False, True),
    ("out_dgrad", 768, 768, EPI_NONE, False, True),
    ("qkv_dgrad+resid", 768, 2304, EPI_RESID, False, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--M", type=int, default=98304)
    a = ap.parse_args()
    k = _native.kernels()
    dev = torch.device("cuda", 0)
    M = a.M
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K, epi, q8, wo in SHAPES:
        grad = epi in (EPI_NONE, EPI_RESID, EPI_DMUL)
        A8 = (torch.randn(M, K, device=dev, generator=g) * 4).to(torch.float8_e5m2 if grad else torch.float8_e4m3fn)
        B8 = (torch.randn(N, K, device=dev, generator=g) * 4).to(torch.float8_e4m3fn)
        one = torch.ones(1, device=dev)
        bias = torch.zeros(N, device=dev)
        kw = {}
        if epi in (EPI_GELUD, EPI_DMUL):
            kw["pre"] = torch.rand(M, N, device=dev, generator=g).bfloat16()
        if epi == EPI_RESID:
            kw["resid"] = torch.rand(M, N, device=dev, generator=g).bfloat16()
        if epi == EPI_DMUL:
            kw["part"] = torch.empty(M // 256, N, device=dev)
        if q8:
            kw["out8"] = torch.empty(M, N, device=dev, dtype=torch.float8_e5m2 if epi == EPI_DMUL else torch.float8_e4m3fn)
            kw["state"] = torch.tensor([0.0, 0.0, 100.0, 0.0], device=dev)
            kw["phase"] = 0
            kw["write_out"] = wo

        def run():
            return k.gemm_fp8(A8, B8, epi, None if grad else bias, one, one, **kw)
        times = {2: [], 3: []}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for v in (2, 3):
                k.gemm_fp8_set_variant(v)
                run()
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) * 1000 / 5)
        k.gemm_fp8_set_variant(0)
        flop = 2.0 * M * N * K
        med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
        print(f"{name:24s} N={N:5d} K={K:5d}  v2 {med[2]:7.1f} us ({flop / med[2] / 1e6:6.0f} TF/s)   "
              f"persistent {med[3]:7.1f} us ({flop / med[3] / 1e6:6.0f} TF/s)   x{med[2] / med[3]:.3f}", flush=True)


if __name__ == "__main__":
    main()
