"""The torch reference ops (CPU path + GPU oracle) against plain autograd of the textbook formulas."""
import math

import pytest
import torch
import torch.nn.functional as F

from ml_recipe_distributed_pytorch_amd.ops import reference as R
from ml_recipe_distributed_pytorch_amd.ops import rng


def _keep(shape, seed, opid, p):
    return rng.keep_mask(shape, seed, opid, p).double() * rng.keep_scale(p)


@pytest.mark.parametrize("p", [0.0, 0.1, 0.5])
def test_rng_mask_statistics(p):
    m = rng.keep_mask((64, 4096), 7, 3, p)
    frac = m.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01
    assert torch.equal(m, rng.keep_mask((64, 4096), 7, 3, p))
    if p > 0:
        assert not torch.equal(m, rng.keep_mask((64, 4096), 7, 4, p))
        assert not torch.equal(m, rng.keep_mask((64, 4096), 8, 3, p))
        # dropout is unbiased in expectation
        assert abs(m.float().mean().item() * rng.keep_scale(p) - 1) < 0.02


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_ln_fwd_bwd(p):
    torch.manual_seed(0)
    T, H, eps, seed, opid = 37, 96, 1e-12, 11, 5
    a = torch.randn(T, H, dtype=torch.float64, requires_grad=True)
    r = torch.randn(T, H, dtype=torch.float64, requires_grad=True)
    gamma = torch.randn(H, dtype=torch.float64, requires_grad=True)
    beta = torch.randn(H, dtype=torch.float64, requires_grad=True)
    keep = _keep((T, H), seed, opid, p) if p > 0 else torch.ones(T, H, dtype=torch.float64)
    z = a * keep + r
    y = F.layer_norm(z, (H,), gamma, beta, eps)
    dy, dy2 = torch.randn(T, H, dtype=torch.float64), torch.randn(T, H, dtype=torch.float64)
    (y * (dy + dy2)).sum().backward()

    y_r, z_r, mean, rstd = R.ln_fwd(a.detach().float(), r.detach().float(), gamma.detach().float(),
                                    beta.detach().float(), eps, p, seed, opid)
    torch.testing.assert_close(y_r.double(), y.detach(), atol=1e-4, rtol=1e-4)
    gg, gb, gbias = torch.zeros(H), torch.zeros(H), torch.zeros(H)
    dz, da = R.ln_bwd(dy.float(), dy2.float(), z_r, gamma.detach().float(), mean, rstd, p, seed, opid, gg, gb, gbias,
                      False)
    torch.testing.assert_close(dz.double(), r.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(da.double(), a.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gg.double(), gamma.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(gb.double(), beta.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(gbias.double(), a.grad.sum(0), atol=1e-3, rtol=1e-4)
    # accumulate=True adds
    R.ln_bwd(dy.float(), dy2.float(), z_r, gamma.detach().float(), mean, rstd, p, seed, opid, gg, gb, gbias, True)
    torch.testing.assert_close(gb.double(), 2 * beta.grad, atol=1e-3, rtol=1e-4)


def test_gelu():
    x = torch.randn(50, 70, dtype=torch.float64, requires_grad=True)
    y = F.gelu(x)
    d = torch.randn_like(y)
    (y * d).sum().backward()
    torch.testing.assert_close(R.gelu_fwd(x.detach().float()).double(), y.detach(), atol=1e-6, rtol=1e-5)
    gb = torch.zeros(70)
    g = R.gelu_bwd(d.float(), x.detach().float(), gb, False)
    torch.testing.assert_close(g.double(), x.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(gb.double(), x.grad.sum(0), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention(p):
    torch.manual_seed(1)
    B, L, nh, dh = 2, 19, 3, 8
    H = nh * dh
    seed, opid, scale = 5, 2, 1 / math.sqrt(dh)
    qkv = torch.randn(B * L, 3 * H, dtype=torch.float64, requires_grad=True)
    mask = torch.ones(B, L)
    mask[1, 13:] = 0
    kb = (1 - mask) * -10000.0
    q, k, v = qkv.view(B, L, 3, nh, dh).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) * scale + kb.double()[:, None, None, :]
    P = torch.softmax(s, -1)
    if p > 0:
        P = P * _keep((B, nh, L, L), seed, opid, p)
    o = (P @ v).permute(0, 2, 1, 3).reshape(B * L, H)
    do = torch.randn_like(o)
    (o * do).sum().backward()
    ctx, lse = R.attn_fwd(qkv.detach().float(), kb, B, L, nh, p, seed, opid, scale)
    torch.testing.assert_close(ctx.double(), o.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(lse.double(), torch.logsumexp(s.detach(), -1), atol=1e-5, rtol=1e-5)
    g = R.attn_bwd(do.float(), qkv.detach().float(), ctx, lse, kb, B, L, nh, p, seed, opid, scale)
    torch.testing.assert_close(g.double(), qkv.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("pad_pos", [-1, 1])
def test_embedding(pad_pos):
    torch.manual_seed(2)
    V, P, Tv, H, T, eps, p, seed = 50, 20, 2, 32, 40, 1e-12, 0.1, 9
    ww = torch.randn(V, H, dtype=torch.float64, requires_grad=True)
    wp = torch.randn(P, H, dtype=torch.float64, requires_grad=True)
    wt = torch.randn(Tv, H, dtype=torch.float64, requires_grad=True)
    gamma = torch.randn(H, dtype=torch.float64, requires_grad=True)
    beta = torch.randn(H, dtype=torch.float64, requires_grad=True)
    ids = torch.randint(0, V, (T,))
    ids[:5] = 0
    pos = torch.randint(0, P, (T,))
    tt = torch.randint(0, Tv, (T,))
    x = ww[ids] + wp[pos] + wt[tt]
    y = F.layer_norm(x, (H,), gamma, beta, eps) * _keep((T, H), seed, 0, p)
    dy = torch.randn_like(y)
    (y * dy).sum().backward()
    yr, mean, rstd = R.embed_fwd(ids, pos, tt, ww.detach().float(), wp.detach().float(), wt.detach().float(),
                                 gamma.detach().float(), beta.detach().float(), eps, p, seed, 0, torch.float32)
    torch.testing.assert_close(yr.double(), y.detach(), atol=1e-4, rtol=1e-4)
    gw, gp, gt = torch.zeros(V, H), torch.zeros(P, H), torch.zeros(Tv, H)
    gg, gb = torch.zeros(H), torch.zeros(H)
    R.embed_bwd(dy.float(), ids, pos, tt, ww.detach().float(), wp.detach().float(), wt.detach().float(),
                gamma.detach().float(), mean, rstd, p, seed, 0, gw, gp, gt, gg, gb, False, pad_word=0, pad_pos=pad_pos)
    exp_w = ww.grad.clone()
    exp_w[0] = 0  # padding_idx row gets no gradient (HF nn.Embedding(padding_idx=pad))
    exp_p = wp.grad.clone()
    if pad_pos >= 0:
        exp_p[pad_pos] = 0
    torch.testing.assert_close(gw.double(), exp_w, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gp.double(), exp_p, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gt.double(), wt.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gg.double(), gamma.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(gb.double(), beta.grad, atol=1e-3, rtol=1e-4)


def test_linear_ops():
    x, w, b = torch.randn(9, 6), torch.randn(4, 6), torch.randn(4)
    dy = torch.randn(9, 4)
    torch.testing.assert_close(R.linear_fwd(x, w, b), F.linear(x, w, b))
    torch.testing.assert_close(R.linear_dgrad(dy, w), dy @ w)
    r = torch.randn(9, 6)
    torch.testing.assert_close(R.linear_dgrad_add(dy, w, r), r + dy @ w)
    gw, gb = torch.zeros(4, 6), torch.zeros(4)
    R.linear_wgrad(dy, x, gw, gb, False)
    torch.testing.assert_close(gw, dy.t() @ x)
    torch.testing.assert_close(gb, dy.sum(0))


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_linear_bdr_ln_fwd_cpu_path(p):
    """The fused projection + dropout + residual + LayerNorm op (GPU: EPI_BDR epilogue + z-in LayerNorm)
    falls back on the CPU to linear_fwd → ln_fwd; its z is dropout(x·Wᵀ + b) + resid and y = LN(z)."""
    from ml_recipe_distributed_pytorch_amd import ops
    torch.manual_seed(0)
    T, K, N = 64, 48, 32
    x, w, b = torch.randn(T, K), torch.randn(N, K) * 0.2, torch.randn(N)
    resid = torch.randn(T, N)
    gamma, beta = torch.randn(N) * 0.1 + 1, torch.randn(N) * 0.1
    y, z, mean, rstd = ops.linear_bdr_ln_fwd(x, w, b, None, resid, "out", gamma, beta, 1e-12, p, 1234, 7)
    y2, z2, m2, r2 = R.ln_fwd(R.linear_fwd(x, w, b), resid, gamma, beta, 1e-12, p, 1234, 7)
    assert torch.equal(z, z2) and torch.equal(y, y2) and torch.equal(mean, m2) and torch.equal(rstd, r2)
    if p == 0.0:
        ref = F.layer_norm(x @ w.t() + b + resid, (N,), gamma, beta, 1e-12)
        assert (y - ref).abs().max().item() < 1e-4
