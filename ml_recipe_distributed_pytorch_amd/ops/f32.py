"""``--precision fp32`` on the GPU (the reference's default when Apex is off: ``apex_level=None`` / ``O0`` train in
fp32, ``/root/reference/modules/model/trainer/trainer.py:23-32,128-133,200-204``; ``--finetune`` forces it,
``/root/reference/modules/init.py:88-89``).

Every GEMM-shaped FLOP runs on the own exact-f32 MFMA kernel (``csrc/kernels/gemm_f32.hip``,
``v_mfma_f32_32x32x2_f32``: a k-ordered fp32 fma chain, no reduced-precision inputs): the encoder projections
(forward, dgrad and weight gradient, addressed as strided views — no transposed copies) and the attention's
batched QKᵀ, PV and their four backward products.  The row-wise / elementwise parts (embedding gathers, LayerNorm,
softmax, GELU, dropout masks from ``ops.rng``) are the fp32 oracle ops of ``ops.reference`` on the device — this
mode exists for numerical parity with the reference's fp32 training, not for speed; the bf16 / fp8 paths are the
fused kernels.
"""
from __future__ import annotations

import torch

from . import reference as ref
from .._native import kernels


def active(t: torch.Tensor) -> bool:
    """The fp32 GPU path handles this activation tensor."""
    return t.is_cuda and t.dtype == torch.float32


def _gemm(A, B, C, M, N, K, sa, sb, sc, batch=1, nb_in=1, alpha=1.0, bias=None, R=None, ldr=0):
    kernels().gemm_f32(A, B, C, int(M), int(N), int(K), [int(v) for v in sa], [int(v) for v in sb],
                       [int(v) for v in sc], int(batch), int(nb_in), float(alpha), bias, R, int(ldr))
    return C


# ------------------------------------------------------------------------------------------------- linear
def linear_fwd(x, w, b):
    """y[M, N] = x[M, K]·w[N, K]ᵀ + b."""
    x, w = x.contiguous(), w.contiguous()
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, dtype=torch.float32, device=x.device)
    return _gemm(x, w, y, M, N, K, (K, 1, 0, 0), (K, 1, 0, 0), (N, 0, 0),
                 bias=None if b is None else b.float().contiguous())


def linear_dgrad(dy, w, resid=None):
    """dx[M, Kin] = dy[M, N]·w[N, Kin] (+ resid): w is read as B(j = kin, k = n) = w[n·Kin + kin]."""
    dy, w = dy.contiguous(), w.contiguous()
    M, N = dy.shape
    Kin = w.shape[1]
    dx = torch.empty(M, Kin, dtype=torch.float32, device=dy.device)
    r = None if resid is None else resid.contiguous()
    return _gemm(dy, w, dx, M, Kin, N, (N, 1, 0, 0), (1, Kin, 0, 0), (Kin, 0, 0), R=r, ldr=Kin)


def linear_wgrad(dy, x, g_w, g_b, accumulate: bool):
    """g_w[N, K] (+)= Σ_m dy[m, n]·x[m, k] straight into the fp32 arena view (split-K, deterministic);
    g_b (+)= column sums of dy."""
    dy, x = dy.contiguous(), x.contiguous()
    T, N = dy.shape
    K = x.shape[1]
    assert g_w.is_contiguous() and g_w.shape == (N, K)
    _gemm(dy, x, g_w, N, K, T, (1, N, 0, 0), (1, K, 0, 0), (K, 0, 0), R=g_w if accumulate else None, ldr=K)
    if g_b is not None:
        ref._acc(g_b, dy.sum(0), accumulate)


# ---------------------------------------------------------------------------------------------- attention
# qkv [T = B·L, 3H] holds q | k | v, head h in columns h·dh … of each third; batch index z = b·nh + h.
def attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale):
    qkv = qkv.contiguous()
    T, H3 = qkv.shape
    H = H3 // 3
    dh = H // nh
    dev = qkv.device
    s = torch.empty(B, nh, L, L, dtype=torch.float32, device=dev)
    # S = scale·Q·Kᵀ: A(i = query, k = d) = qkv[(bL + i)·3H + h·dh + d], B(j = key, k = d) = qkv[… + H + …]
    _gemm(qkv, qkv[:, H:], s, L, L, dh, (H3, 1, L * H3, dh), (H3, 1, L * H3, dh), (L, nh * L * L, L * L),
          batch=B * nh, nb_in=nh, alpha=scale)
    s += key_bias.float()[:, None, None, :]
    lse = torch.logsumexp(s, -1)
    P = torch.exp(s - lse[..., None])
    keep = ref._attn_keep(B, nh, L, seed, opid, p, dev)
    if keep is not None:
        P = P * keep
    ctx = torch.empty(T, H, dtype=torch.float32, device=dev)
    # O = P·V: A(i, k = key) = P[z][i·L + k], B(j = d, k = key) = qkv[(bL + k)·3H + 2H + h·dh + d]
    _gemm(P, qkv[:, 2 * H:], ctx, L, dh, L, (L, 1, nh * L * L, L * L), (1, H3, L * H3, dh), (H, L * H, dh),
          batch=B * nh, nb_in=nh)
    return ctx, lse


def attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale):
    qkv, dctx, ctx = qkv.contiguous(), dctx.contiguous(), ctx.contiguous()
    T, H3 = qkv.shape
    H = H3 // 3
    dh = H // nh
    dev = qkv.device
    bat = dict(batch=B * nh, nb_in=nh)
    sq = (nh * L * L, L * L)                     # batch strides of a [B, nh, L, L] tensor
    s = torch.empty(B, nh, L, L, dtype=torch.float32, device=dev)
    _gemm(qkv, qkv[:, H:], s, L, L, dh, (H3, 1, L * H3, dh), (H3, 1, L * H3, dh), (L,) + sq, alpha=scale, **bat)
    s += key_bias.float()[:, None, None, :]
    P = torch.exp(s - lse[..., None])
    del s
    keep = ref._attn_keep(B, nh, L, seed, opid, p, dev)
    Pd = P * keep if keep is not None else P
    dqkv = torch.empty(T, H3, dtype=torch.float32, device=dev)
    # dV[k, d] = Σ_q Pd[q, k]·dO[q, d]: A(i = k, kk = q) = Pd[q·L + k] (i-contiguous), B(j = d, kk = q) = dO
    _gemm(Pd, dctx, dqkv[:, 2 * H:], L, dh, L, (1, L) + sq, (1, H, L * H, dh), (H3, L * H3, dh), **bat)
    del Pd
    # dP[q, k] = Σ_d dO[q, d]·V[k, d]
    dP = torch.empty(B, nh, L, L, dtype=torch.float32, device=dev)
    _gemm(dctx, qkv[:, 2 * H:], dP, L, L, dh, (H, 1, L * H, dh), (H3, 1, L * H3, dh), (L,) + sq, **bat)
    if keep is not None:
        dP = dP * keep
    delta = (dctx.view(B, L, nh, dh) * ctx.view(B, L, nh, dh)).sum(-1).permute(0, 2, 1)   # [B, nh, L]
    dS = P * (dP - delta[..., None])
    del dP, P
    # dQ = scale·dS·K: A = dS (k-contiguous), B(j = d, kk = key) = K[(bL + key)·3H + H + h·dh + d]
    _gemm(dS, qkv[:, H:], dqkv, L, dh, L, (L, 1) + sq, (1, H3, L * H3, dh), (H3, L * H3, dh), alpha=scale, **bat)
    # dK = scale·dSᵀ·Q: A(i = key, kk = q) = dS[q·L + key] (i-contiguous), B(j = d, kk = q) = Q
    _gemm(dS, qkv, dqkv[:, H:], L, dh, L, (1, L) + sq, (1, H3, L * H3, dh), (H3, L * H3, dh), alpha=scale, **bat)
    return dqkv
