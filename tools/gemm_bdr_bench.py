import sys, os, statistics, torch
sys.path.insert(0, os.getcwd())
from ml_recipe_distributed_pytorch_amd import _native
k = _native.kernels(); dev = torch.device("cuda", 0)
M = 98304
for (N, K) in ((768, 3072), (768, 768)):
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16(); B = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
    b = torch.rand(N, device=dev); R = torch.randn(M, N, device=dev).bfloat16(); C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res = {}
    for _ in range(9):
        for v in (0, 2, 3):
            for epi in (1, 7):
                k.gemm_set_variant(v)
                kw = dict(bias=b, out=C)
                if epi == 7: kw.update(resid=R, p=0.1, seed=1, opid=3)
                torch.cuda.synchronize(); e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(); k.gemm_nt(A, B, epi, **kw); e1.record(); torch.cuda.synchronize()
                res.setdefault((v, epi), []).append(e0.elapsed_time(e1) * 1e3)
    k.gemm_set_variant(0)
    for key, vals in sorted(res.items()):
        print(f"N={N} K={K} variant={key[0]} epi={'bias' if key[1]==1 else 'bdr'}: {statistics.median(vals):.1f} us")
