#!/usr/bin/env python
"""Run one NT GEMM shape repeatedly (for PMC collection): python tools/gemm_one.py T N K epi
(optional 5th argument: kernel variant for gemm_set_variant, e.g. 1 = v1)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402

T, N, K, epi = (int(x) for x in sys.argv[1:5])
k = _native.kernels()
k.gemm_set_variant(int(sys.argv[5]) if len(sys.argv) > 5 else 0)
dev = torch.device("cuda")
A = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
bias = torch.rand(N, device=dev)
C = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
for _ in range(10):
    k.gemm_nt(A, B, epi, bias=bias if epi == 1 else None, out=C)
torch.cuda.synchronize()
print("ok")
