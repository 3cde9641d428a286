"""Context only (never used by the framework): the vendor library's time on the headline GEMM shapes, next to
the in-tree kernels, same box / same inputs.  Prints µs and PF/s per shape; run under rocprofv3 to see the
vendor kernel names (their tile configuration)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

k = _native.kernels()
dev = torch.device("cuda", 0)
T = 256 * 384
SHAPES = [("qkv fwd", T, 2304, 768), ("attn-out fwd", T, 768, 768), ("ffn1 fwd", T, 3072, 768),
          ("ffn2 fwd", T, 768, 3072)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / n


for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    fl = 2.0 * M * N * K
    tv = timeit(lambda: torch.matmul(a, b.t()))
    to = timeit(lambda: k.gemm_nt(a, b, 0))
    # weight gradient shape: [N, K] = dyᵀ · x over T tokens
    dy = torch.randn(M, N, device=dev).bfloat16()
    out = torch.zeros(N, K, device=dev)
    tvw = timeit(lambda: torch.matmul(dy.t(), a))
    tow = timeit(lambda: k.gemm_tn(dy, a, out, False, 0, None))
    print(f"{name:13s} M={M} N={N} K={K}: nt vendor {tv:7.1f} us ({fl / tv / 1e9:.2f} PF) own {to:7.1f} us "
          f"({fl / to / 1e9:.2f} PF) | wgrad vendor {tvw:7.1f} us ({fl / tvw / 1e9:.2f} PF) own {tow:7.1f} us "
          f"({fl / tow / 1e9:.2f} PF)", flush=True)
