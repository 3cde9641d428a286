"""``--precision fp32`` on the GPU (the reference's default when Apex is off: ``apex_level=None`` / ``O0`` train in
fp32, ``/root/reference/modules/model/trainer/trainer.py:23-32,128-133,200-204``; ``--finetune`` forces it,
``/root/reference/modules/init.py:88-89``).

Every GEMM-shaped FLOP runs on the own exact-f32 MFMA kernel (``csrc/kernels/gemm_f32.hip``,
``v_mfma_f32_32x32x2_f32``: a k-ordered fp32 fma chain, no reduced-precision inputs): the encoder projections
(forward, dgrad and weight gradient, addressed as strided views — no transposed copies).  The attention is a
flash-style fp32 kernel (``csrc/kernels/f32_ops.hip``: scores recomputed per 32-key tile in registers, online
softmax forward, LSE backward — no [B, nh, L, L] tensor at any length), and the row-wise / elementwise parts
(embedding gathers + LayerNorm, residual + dropout + LayerNorm, GELU, the bias-gradient column sums) are own fp32
kernels too, with the dropout masks of ``ops.rng`` — so the fp32 GPU model reproduces the CPU oracle op for op.
This mode exists for numerical parity with the reference's fp32 training; the bf16 / fp8 paths are the fast ones.
"""
from __future__ import annotations

import torch

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
        kernels().f32_colsum(dy, g_b, bool(accumulate))


# ------------------------------------------------------------------------------------ row-wise ops (f32_ops.hip)
def embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid):
    return tuple(kernels().f32_embed_fwd(ids.contiguous(), pos_ids.contiguous(), type_ids.contiguous(),
                                         w_word.contiguous(), w_pos.contiguous(), w_type.contiguous(), gamma.contiguous(),
                                         beta.contiguous(), float(eps), float(p), int(seed), int(opid)))


def embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
              g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word=-1, pad_pos=-1):
    kernels().f32_embed_bwd(dy.contiguous(), ids.contiguous(), pos_ids.contiguous(), type_ids.contiguous(),
                            w_word.contiguous(), w_pos.contiguous(), w_type.contiguous(), gamma.contiguous(), mean, rstd,
                            float(p), int(seed), int(opid), g_word, g_pos, g_type, g_gamma, g_beta, bool(accumulate),
                            int(pad_word), int(pad_pos))


def ln_fwd(a, resid, gamma, beta, eps, p, seed, opid):
    """z = dropout(a) + resid, y = LN(z): (y, z, mean, rstd)."""
    return tuple(kernels().f32_ln_fwd(a.contiguous(), resid.contiguous(), gamma.contiguous(), beta.contiguous(),
                                      float(eps), float(p), int(seed), int(opid)))


def ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate, beta=None):
    return tuple(kernels().f32_ln_bwd(dy.contiguous(), None if dy2 is None else dy2.contiguous(), z.contiguous(),
                                      gamma.contiguous(), mean, rstd, float(p), int(seed), int(opid), g_gamma, g_beta,
                                      g_bias, bool(accumulate), beta=None if beta is None else beta.contiguous()))


# ---------------------------------------------------------------------------------------------- attention
# qkv [T = B·L, 3H] holds q | k | v, head h in columns h·dh … of each third; batch index z = b·nh + h.
def attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale):
    """(ctx [T, H], lse [B, nh, L]) from the flash fp32 kernel (head_dim 64)."""
    ctx, lse = kernels().f32_attn_fwd(qkv.contiguous(), key_bias.float().contiguous(), int(B), int(L), int(nh), float(p),
                                      int(seed), int(opid), float(scale))
    return ctx, lse


def attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale):
    """dQKV [T, 3H]: a dQ kernel (which also writes δ = rowsum(dO ∘ O)) and a dK / dV kernel, both recomputing P
    from the forward's LSE and the dropout keep bits from the hash."""
    return kernels().f32_attn_bwd(dctx.contiguous(), qkv.contiguous(), ctx.contiguous(), lse.contiguous(),
                                  key_bias.float().contiguous(), int(B), int(L), int(nh), float(p), int(seed), int(opid),
                                  float(scale))
