"""Debug: v3 persistent GEMM epilogues vs fp32 reference, halftail on/off; prints where outputs go wrong."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

k = _native.kernels()
dev = torch.device("cuda", 0)
M, N, K = [int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (98304, 768, 768))]
g = torch.Generator(device=dev).manual_seed(M + K)
A = (torch.randn(M, K, device=dev, generator=g) * 0.5).bfloat16()
B = (torch.randn(N, K, device=dev, generator=g) * 0.1).bfloat16()
bias = torch.randn(N, device=dev, generator=g) * 0.1
ref = A.float() @ B.float().t()
HT = 1 << 16
for epi in (1, 2, 5):
    for w in (0, HT):
        k.gemm_set_stagger(w)
        pre = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        o = k.gemm_nt(A, B, epi, bias=bias, pre=pre) if epi != 1 else k.gemm_nt(A, B, epi, bias=bias)
        torch.cuda.synchronize()
        x = (ref + bias)
        exp = x if epi == 1 else torch.nn.functional.gelu(x.bfloat16().float())
        err = (o.float() - exp).abs()
        bad = err > 0.05 * (exp.abs().max())
        nb = int(bad.sum())
        msg = f"epi {epi} ht {w>>16}: bad {nb}"
        if nb:
            r, c = torch.nonzero(bad, as_tuple=True)
            msg += f" rows {int(r.min())}..{int(r.max())} (distinct {len(torch.unique(r // 128))} 128-blocks) cols {int(c.min())}..{int(c.max())}"
            msg += f" nan {int(torch.isnan(o.float()).sum())}"
        if epi != 1:
            perr = ((pre.float() - x).abs() > 0.05 * x.abs().max())
            msg += f" | pre bad {int(perr.sum())} nan {int(torch.isnan(pre.float()).sum())}"
            if int(perr.sum()):
                r, c = torch.nonzero(perr, as_tuple=True)
                msg += f" col%8 {torch.bincount(c % 8, minlength=8).tolist()}"
                msg += f" row%16 {torch.bincount(r % 16, minlength=16).tolist()}"
                msg += f" col%128//8 {torch.bincount((c % 128) // 8, minlength=16).tolist()}"
                msg += f" tiles {len(torch.unique((r // 256) * 64 + c // 256))}"
        if nb:
            r, c = torch.nonzero(bad, as_tuple=True)
            msg += f" || C col%8 {torch.bincount(c % 8, minlength=8).tolist()}"
        print(msg, flush=True)
k.gemm_set_stagger(HT)
