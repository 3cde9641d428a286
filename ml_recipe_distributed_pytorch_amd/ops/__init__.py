"""Fused-op API used by the model.  Dispatch is by device, not by a backend registry:

* CUDA (ROCm/HIP) tensors → hand-written gfx950 kernels in ``_hq_kernels.so`` (fail loudly if absent);
  plain GEMMs go to hipBLASLt through ``torch.addmm/mm`` (library GEMMs, no fused epilogue needed).
* CPU tensors → ``ops.reference`` (pure PyTorch, fp32), which is also the numerics oracle.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref
from . import rng  # noqa: F401
from .._native import kernels


def _k():
    return kernels()


# ------------------------------------------------------------------------------------ embedding
def embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid, out_dtype):
    if ids.is_cuda:
        return tuple(_k().embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta,
                                    float(eps), float(p), int(seed), int(opid)))
    return ref.embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid, out_dtype)


def embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
              g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word=-1, pad_pos=-1):
    if dy.is_cuda:
        return _k().embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, float(p),
                              int(seed), int(opid), g_word, g_pos, g_type, g_gamma, g_beta, bool(accumulate),
                              int(pad_word), int(pad_pos))
    return ref.embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
                         g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word, pad_pos)


# ------------------------------------------------------------------ residual + dropout + LayerNorm
def ln_fwd(a, resid, gamma, beta, eps, p, seed, opid):
    if a.is_cuda:
        return tuple(_k().ln_fwd(a, resid, gamma, beta, float(eps), float(p), int(seed), int(opid)))
    return ref.ln_fwd(a, resid, gamma, beta, eps, p, seed, opid)


def ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate):
    if dy.is_cuda:
        return tuple(_k().ln_bwd(dy, dy2, z, gamma, mean, rstd, float(p), int(seed), int(opid),
                                 g_gamma, g_beta, g_bias, bool(accumulate)))
    return ref.ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate)


# ------------------------------------------------------------------------------------------ GELU
def gelu_fwd(pre):
    if pre.is_cuda:
        return _k().gelu_fwd(pre)
    return ref.gelu_fwd(pre)


def gelu_bwd(dout, pre, g_bias, accumulate):
    if dout.is_cuda:
        return _k().gelu_bwd(dout, pre, g_bias, bool(accumulate))
    return ref.gelu_bwd(dout, pre, g_bias, accumulate)


# ------------------------------------------------------------------------------------- attention
def attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale):
    if qkv.is_cuda:
        return tuple(_k().attn_fwd(qkv, key_bias, int(B), int(L), int(nh), float(p), int(seed), int(opid),
                                   float(scale)))
    return ref.attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale)


def attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale):
    if dctx.is_cuda:
        return _k().attn_bwd(dctx, qkv, ctx, lse, key_bias, int(B), int(L), int(nh), float(p), int(seed),
                             int(opid), float(scale))
    return ref.attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale)


# --------------------------------------------------------------------------------------- linear
def linear_fwd(x, w, b):
    """y = x·Wᵀ + b — hipBLASLt GEMM with its bias epilogue on GPU."""
    if x.is_cuda:
        return torch.addmm(b, x, w.t()) if b is not None else torch.mm(x, w.t())
    return ref.linear_fwd(x, w, b)


def linear_dgrad(dy, w):
    if dy.is_cuda:
        return torch.mm(dy, w)
    return ref.linear_dgrad(dy, w)


def linear_dgrad_add(dy, w, resid):
    """resid + dy·W (hipBLASLt beta=1 accumulate; fuses the residual-gradient add)."""
    if dy.is_cuda:
        return torch.addmm(resid, dy, w)
    return ref.linear_dgrad_add(dy, w, resid)


def linear_wgrad(dy, x, g_w, g_b, accumulate):
    """g_w (fp32 arena view) (+)= dyᵀ·x with fp32 GEMM output; g_b (+)= column sums of dy."""
    if dy.is_cuda:
        if accumulate:
            g_w.add_(torch.mm(dy.t(), x, out_dtype=torch.float32))
        else:
            torch.mm(dy.t(), x, out_dtype=torch.float32, out=g_w)
        if g_b is not None:
            _k().bias_grad(dy, g_b, bool(accumulate))
        return
    ref.linear_wgrad(dy, x, g_w, g_b, accumulate)


def bias_grad(dy, g_b, accumulate):
    if dy.is_cuda:
        return _k().bias_grad(dy, g_b, bool(accumulate))
    ref._acc(g_b, dy.float().sum(0), accumulate)
