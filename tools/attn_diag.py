"""Debug: where does the attention backward differ from the fp32 oracle (tests/test_kernels_gpu.py::_attn_case)?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from ml_recipe_distributed_pytorch_amd import _native  # noqa: E402
from ml_recipe_distributed_pytorch_amd.ops import reference as ref  # noqa: E402

k = _native.kernels()
cuda = torch.device("cuda", 0)
for ramp in (0.3, 0.05, 0.0):
    B, L, nh, p = 2, 384, 2, 0.1
    torch.manual_seed(3)
    H = nh * 64
    bf = lambda t: t.bfloat16()  # noqa: E731
    qkv = bf(torch.randn(B * L, 3 * H))
    kb = ramp * torch.arange(L, dtype=torch.float32).expand(B, L).clone()
    for b in range(B):
        kb[b, L - 1 - 7 * b:] = -10000.0
    scale = 1.0 / 8.0
    ctx, lse, bits = k.attn_fwd(qkv.to(cuda), kb.to(cuda), B, L, nh, p, 555, 3, scale)
    dctx = bf(torch.randn(B * L, H))
    dq = k.attn_bwd(dctx.to(cuda), qkv.to(cuda), ctx, lse, kb.to(cuda), bits, B, L, nh, p, scale, False)
    dqr = ref.attn_bwd(dctx, qkv, ctx.cpu(), lse.cpu(), kb, B, L, nh, p, 555, 3, scale)
    a, r = dq.float().cpu(), dqr.float()
    err = (a - r).abs()
    rel = err / (0.03 + 0.03 * r.abs())
    for sec, name in enumerate("QKV"):
        e = rel[:, sec * H:(sec + 1) * H]
        i = int(e.argmax())
        t, c = divmod(i, H)
        print(f"ramp {ramp} d{name}: worst tol-ratio {float(e.max()):.3f} at token {t} col {c}: got "
              f"{float(a[t, sec * H + c]):.5f} ref {float(r[t, sec * H + c]):.5f}; max abs err "
              f"{float(err[:, sec * H:(sec + 1) * H].max()):.4f}", flush=True)
