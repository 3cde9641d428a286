"""The native fp32 row-wise ops and flash attention of ``--precision fp32`` (csrc/kernels/f32_ops.hip) against the
fp32 CPU oracle (ops/reference.py) — same inputs, same dropout masks (ops.rng counter hash)."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native
from ml_recipe_distributed_pytorch_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, tol, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = float((a - b).abs().max())
    scale = float(b.abs().max()) + 1e-12
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("B,L,nh,p", [(2, 77, 2, 0.0), (2, 77, 2, 0.1), (3, 128, 4, 0.1), (1, 5, 1, 0.1), (2, 200, 12, 0.1)])
def test_f32_attention_matches_oracle(cuda, B, L, nh, p):
    """Flash fp32 forward (online softmax over 32-key tiles, L not a multiple of the tile) and backward (dQ + δ,
    then dK / dV) vs the materialised-L×L oracle, with a padded key block and dropout."""
    k = _native.kernels()
    g = torch.Generator().manual_seed(L + nh)
    H = 64 * nh
    qkv = torch.randn(B * L, 3 * H, generator=g)
    mask = torch.ones(B, L, dtype=torch.bool)
    mask[0, L - L // 4:] = False
    kb = (1.0 - mask.float()) * -10000.0
    scale = 0.125
    ctx, lse = k.f32_attn_fwd(qkv.to(cuda), kb.to(cuda), B, L, nh, p, 7, 3, scale)
    rctx, rlse = ref.attn_fwd(qkv, kb, B, L, nh, p, 7, 3, scale)
    _close(ctx, rctx, 2e-5, "ctx")
    _close(lse, rlse, 1e-5, "lse")
    dctx = torch.randn(B * L, H, generator=g)
    dqkv = k.f32_attn_bwd(dctx.to(cuda), qkv.to(cuda), ctx, lse, kb.to(cuda), B, L, nh, p, 7, 3, scale)
    rd = ref.attn_bwd(dctx, qkv, rctx, rlse, kb, B, L, nh, p, 7, 3, scale)
    for i, n in enumerate(("dq", "dk", "dv")):
        _close(dqkv[:, i * H:(i + 1) * H], rd[:, i * H:(i + 1) * H], 5e-5, n)


@pytest.mark.parametrize("H", [768, 128])
@pytest.mark.parametrize("from_y", [False, True])
def test_f32_layernorm_matches_oracle(cuda, H, from_y):
    k = _native.kernels()
    g = torch.Generator().manual_seed(H)
    T = 300
    a, r = torch.randn(T, H, generator=g), torch.randn(T, H, generator=g)
    gamma, beta = torch.randn(H, generator=g) * 0.3 + 1, torch.randn(H, generator=g) * 0.1
    y, z, m, rs = k.f32_ln_fwd(a.to(cuda), r.to(cuda), gamma.to(cuda), beta.to(cuda), 1e-12, 0.1, 5, 2)
    ry, rz, rm, rr = ref.ln_fwd(a, r, gamma, beta, 1e-12, 0.1, 5, 2)
    _close(y, ry, 1e-5, "y"); _close(z, rz, 1e-6, "z"); _close(m, rm, 1e-5, "mean"); _close(rs, rr, 1e-5, "rstd")
    dy, dy2 = torch.randn(T, H, generator=g), torch.randn(T, H, generator=g)
    outs = [torch.randn(H, generator=g) for _ in range(3)]
    gg = [o.to(cuda) for o in outs]
    zin = y if from_y else z
    dz, da = k.f32_ln_bwd(dy.to(cuda), dy2.to(cuda), zin, gamma.to(cuda), m, rs, 0.1, 5, 2, *gg, True,
                          beta=beta.to(cuda) if from_y else None)
    rg = [o.clone() for o in outs]
    rdz, rda = ref.ln_bwd(dy, dy2, (ry if from_y else rz), gamma, rm, rr, 0.1, 5, 2, *rg, True,
                          beta=beta if from_y else None)
    _close(dz, rdz, 5e-5, "dz"); _close(da, rda, 5e-5, "da")
    for x, y_, n in zip(gg, rg, ("g_gamma", "g_beta", "g_bias")):
        _close(x, y_, 1e-5, n)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_f32_embedding_matches_oracle(cuda, p):
    k = _native.kernels()
    g = torch.Generator().manual_seed(3)
    V, P, H, B, L = 500, 64, 768, 3, 40
    T = B * L
    ww, wp, wt = (torch.randn(V, H, generator=g) * 0.05, torch.randn(P, H, generator=g) * 0.05,
                  torch.randn(2, H, generator=g) * 0.05)
    gamma, beta = torch.randn(H, generator=g) * 0.3 + 1, torch.randn(H, generator=g) * 0.1
    ids = torch.randint(0, V, (T,), generator=g)
    ids[::9] = 0
    pids = torch.arange(L).repeat(B)
    tids = torch.randint(0, 2, (T,), generator=g)
    dev = lambda t: t.to(cuda)  # noqa: E731
    y, m, rs = k.f32_embed_fwd(dev(ids), dev(pids), dev(tids), dev(ww), dev(wp), dev(wt), dev(gamma), dev(beta), 1e-12, p,
                               9, 1)
    ry, rm, rr = ref.embed_fwd(ids, pids, tids, ww, wp, wt, gamma, beta, 1e-12, p, 9, 1, torch.float32)
    _close(y, ry, 1e-5, "y")
    dy = torch.randn(T, H, generator=g)
    outs = [torch.randn(V, H, generator=g), torch.randn(P, H, generator=g), torch.randn(2, H, generator=g),
            torch.randn(H, generator=g), torch.randn(H, generator=g)]
    for acc in (False, True):
        go = [dev(o.clone()) for o in outs]
        k.f32_embed_bwd(dev(dy), dev(ids), dev(pids), dev(tids), dev(ww), dev(wp), dev(wt), dev(gamma), m, rs, p, 9, 1,
                        *go, acc, 0, -1)
        ro = [o.clone() for o in outs]
        ref.embed_bwd(dy, ids, pids, tids, ww, wp, wt, gamma, rm, rr, p, 9, 1, *ro, acc, 0, -1)
        for a, b, n in zip(go, ro, ("word", "pos", "type", "gamma", "beta")):
            _close(a, b, 1e-5, f"{n} (accumulate={acc})")


def test_f32_gelu_and_colsum_match_oracle(cuda):
    k = _native.kernels()
    g = torch.Generator().manual_seed(4)
    x, dout = torch.randn(333, 3072, generator=g) * 2, torch.randn(333, 3072, generator=g)
    _close(k.f32_gelu_fwd(x.to(cuda)), ref.gelu_fwd(x), 1e-6, "gelu")
    gb = torch.randn(3072, generator=g)
    gd = gb.to(cuda)
    d = k.f32_gelu_bwd(dout.to(cuda), x.to(cuda), gd, True)
    rgb = gb.clone()
    rd = ref.gelu_bwd(dout, x, rgb, True)
    _close(d, rd, 1e-6, "dgelu")
    _close(gd, rgb, 1e-5, "bias grad")
    out = torch.zeros(3072, device=cuda)
    k.f32_colsum(dout.to(cuda), out, False)
    _close(out, dout.double().sum(0), 1e-5, "colsum")
