"""Pure-PyTorch implementations of every fused op (CPU path + numerics oracle).

Each function has the same signature and the same side effects (grad accumulation into fp32
arena views) as its HIP kernel twin in ``csrc/kernels``.  Math is done in fp32; outputs are
cast to the compute dtype of the activations.  Dropout masks come from ``ops.rng`` so the CPU
and GPU paths draw *identical* masks for the same (seed, opid).

Semantics follow HF ``BertModel`` as used by the reference (``modules/model/model/model.py:20-25``):
erf GELU, LayerNorm with fp32 statistics, additive ``-10000`` key mask, dropout after the
embedding LayerNorm, on attention probabilities, and before each residual add.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import rng

Tensor = torch.Tensor


def _acc(dst: Optional[Tensor], val: Tensor, accumulate: bool) -> None:
    if dst is None:
        return
    if accumulate:
        dst.add_(val.to(dst.dtype))
    else:
        dst.copy_(val.to(dst.dtype))


def _drop_keep(shape, seed, opid, p, device):
    if p <= 0.0:
        return None
    return rng.keep_mask(shape, seed, opid, p, device=device).to(torch.float32) * rng.keep_scale(p)


def _ln_stats(x: Tensor, eps: float):
    mean = x.mean(-1)
    var = ((x - mean[:, None]) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    return mean, rstd


def _ln_bwd_core(g: Tensor, xhat: Tensor, gamma: Tensor, rstd: Tensor) -> Tensor:
    dxhat = g * gamma.float()[None, :]
    return rstd[:, None] * (dxhat - dxhat.mean(-1, keepdim=True) - xhat * (dxhat * xhat).mean(-1, keepdim=True))


# ------------------------------------------------------------------------------------ embedding
def embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid, out_dtype):
    x = w_word.float()[ids] + w_pos.float()[pos_ids] + w_type.float()[type_ids]
    mean, rstd = _ln_stats(x, eps)
    y = (x - mean[:, None]) * rstd[:, None] * gamma.float()[None] + beta.float()[None]
    keep = _drop_keep(y.shape, seed, opid, p, y.device)
    if keep is not None:
        y = y * keep
    return y.to(out_dtype), mean, rstd


def embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
              g_word, g_pos, g_type, g_gamma, g_beta, accumulate: bool, pad_word: int = -1, pad_pos: int = -1):
    """``pad_word``/``pad_pos``: rows that receive no gradient (nn.Embedding ``padding_idx``; -1 = none)."""
    x = w_word.float()[ids] + w_pos.float()[pos_ids] + w_type.float()[type_ids]
    xhat = (x - mean[:, None]) * rstd[:, None]
    g = dy.float()
    keep = _drop_keep(g.shape, seed, opid, p, g.device)
    if keep is not None:
        g = g * keep
    _acc(g_gamma, (g * xhat).sum(0), accumulate)
    _acc(g_beta, g.sum(0), accumulate)
    dx = _ln_bwd_core(g, xhat, gamma, rstd)
    for table, idx, pad in ((g_word, ids, pad_word), (g_pos, pos_ids, pad_pos), (g_type, type_ids, -1)):
        if table is None:
            continue
        if not accumulate:
            table.zero_()
        src = dx if pad < 0 else dx * (idx != pad).to(dx.dtype)[:, None]
        table.index_add_(0, idx, src.to(table.dtype))


# ------------------------------------------------------------------ residual + dropout + LayerNorm
def ln_fwd(a, resid, gamma, beta, eps, p, seed, opid):
    """z = dropout(a) + resid ; y = LN(z).  Returns (y, z, mean, rstd)."""
    af = a.float()
    keep = _drop_keep(af.shape, seed, opid, p, af.device)
    if keep is not None:
        af = af * keep
    z = af + resid.float()
    mean, rstd = _ln_stats(z, eps)
    y = (z - mean[:, None]) * rstd[:, None] * gamma.float()[None] + beta.float()[None]
    return y.to(a.dtype), z.to(a.dtype), mean, rstd


def ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate: bool, beta=None):
    """Returns (dz, da): dz = dL/dz (residual grad), da = dropout_bwd(dz) (GEMM-output grad).  With ``beta``,
    ``z`` is the forward output y and x̂ = (y − β)/γ (0 where γ = 0), as the GPU kernel's FROMY form."""
    g = dy.float()
    if dy2 is not None:
        g = g + dy2.float()
    if beta is not None:
        gf = gamma.float()
        ig = torch.where(gf != 0, 1.0 / gf, torch.zeros_like(gf))
        xhat = z.float() * ig[None] - (beta.float() * ig)[None]
    else:
        xhat = (z.float() - mean[:, None]) * rstd[:, None]
    _acc(g_gamma, (g * xhat).sum(0), accumulate)
    _acc(g_beta, g.sum(0), accumulate)
    dz = _ln_bwd_core(g, xhat, gamma, rstd)
    keep = _drop_keep(dz.shape, seed, opid, p, dz.device)
    da = dz * keep if keep is not None else dz
    _acc(g_bias, da.sum(0), accumulate)
    return dz.to(dy.dtype), da.to(dy.dtype)


# ------------------------------------------------------------------------------------------ GELU
_INV_SQRT2 = 1.0 / math.sqrt(2.0)
_INV_SQRT2PI = 1.0 / math.sqrt(2.0 * math.pi)


def gelu_fwd(pre):
    x = pre.float()
    return (0.5 * x * (1.0 + torch.erf(x * _INV_SQRT2))).to(pre.dtype)


def gelu_bwd(dout, pre, g_bias, accumulate: bool):
    x = pre.float()
    d = dout.float() * (0.5 * (1.0 + torch.erf(x * _INV_SQRT2)) + x * torch.exp(-0.5 * x * x) * _INV_SQRT2PI)
    _acc(g_bias, d.sum(0), accumulate)
    return d.to(dout.dtype)


# ------------------------------------------------------------------------------------- attention
def _split_qkv(qkv, B, L, nh):
    H = qkv.shape[1] // 3
    dh = H // nh
    t = qkv.float().view(B, L, 3, nh, dh).permute(2, 0, 3, 1, 4)
    return t[0], t[1], t[2]


def _attn_keep(B, nh, L, seed, opid, p, device):
    return _drop_keep((B, nh, L, L), seed, opid, p, device)


def attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale):
    q, k, v = _split_qkv(qkv, B, L, nh)
    s = torch.matmul(q, k.transpose(-1, -2)) * scale + key_bias.float()[:, None, None, :]
    lse = torch.logsumexp(s, -1)
    P = torch.exp(s - lse[..., None])
    keep = _attn_keep(B, nh, L, seed, opid, p, qkv.device)
    if keep is not None:
        P = P * keep
    o = torch.matmul(P, v)
    T = B * L
    return o.permute(0, 2, 1, 3).reshape(T, -1).to(qkv.dtype), lse


def attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale):
    q, k, v = _split_qkv(qkv, B, L, nh)
    H = qkv.shape[1] // 3
    dh = H // nh
    do = dctx.float().view(B, L, nh, dh).permute(0, 2, 1, 3)
    o = ctx.float().view(B, L, nh, dh).permute(0, 2, 1, 3)
    s = torch.matmul(q, k.transpose(-1, -2)) * scale + key_bias.float()[:, None, None, :]
    P = torch.exp(s - lse[..., None])
    keep = _attn_keep(B, nh, L, seed, opid, p, qkv.device)
    Pd = P * keep if keep is not None else P
    dv = torch.matmul(Pd.transpose(-1, -2), do)
    dP = torch.matmul(do, v.transpose(-1, -2))
    if keep is not None:
        dP = dP * keep
    delta = (do * o).sum(-1, keepdim=True)
    dS = P * (dP - delta)
    dq = torch.matmul(dS, k) * scale
    dk = torch.matmul(dS.transpose(-1, -2), q) * scale
    out = torch.stack([dq, dk, dv], 0)  # [3,B,nh,L,dh]
    return out.permute(1, 3, 0, 2, 4).reshape(B * L, 3 * H).to(dctx.dtype)


# --------------------------------------------------------------------------------------- linear
def linear_fwd(x, w, b):
    y = x.float() @ w.float().t()
    if b is not None:
        y = y + b.float()
    return y.to(x.dtype)


def linear_dgrad(dy, w):
    return (dy.float() @ w.float()).to(dy.dtype)


def linear_dgrad_add(dy, w, resid):
    return (resid.float() + dy.float() @ w.float()).to(dy.dtype)


def linear_wgrad(dy, x, g_w, g_b, accumulate: bool):
    _acc(g_w, dy.float().t() @ x.float(), accumulate)
    if g_b is not None:
        _acc(g_b, dy.float().sum(0), accumulate)


# ------------------------------------------------------------------------------------ optimizer
def grad_sq_norm(grad: Tensor) -> Tensor:
    return (grad.float() ** 2).sum()


def adamw_step(master, compute, grad, exp_avg, exp_avg_sq, segments, *, lr, beta1, beta2, eps,
               clip_coef: Optional[Tensor], correct_bias: bool, step: int):
    """HF ``AdamW`` (decay AFTER the update, reference ``init.py:137``) over flat arena segments.

    ``segments``: list of (start, numel, weight_decay).
    """
    g = grad if clip_coef is None else grad * clip_coef
    for start, numel, wd in segments:
        sl = slice(start, start + numel)
        gg = g[sl]
        m = exp_avg[sl]
        v = exp_avg_sq[sl]
        p = master[sl]
        m.mul_(beta1).add_(gg, alpha=1.0 - beta1)
        v.mul_(beta2).addcmul_(gg, gg, value=1.0 - beta2)
        denom = v.sqrt().add_(eps)
        step_size = lr
        if correct_bias:
            step_size = lr * math.sqrt(1.0 - beta2 ** step) / (1.0 - beta1 ** step)
        p.addcdiv_(m, denom, value=-step_size)
        if wd > 0.0:
            p.add_(p, alpha=-lr * wd)
    if compute is not None and compute.data_ptr() != master.data_ptr():
        for start, numel, _ in segments:
            compute[start:start + numel].copy_(master[start:start + numel])


def adamod_step(master, compute, grad, exp_avg, exp_avg_sq, exp_avg_lr, segments, *, lr, beta1, beta2, beta3,
                eps, clip_coef: Optional[Tensor], step: int):
    """AdaMod (reference ``modules/model/trainer/optim.py:76-98``): decay BEFORE the update."""
    g = grad if clip_coef is None else grad * clip_coef
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    base = lr * math.sqrt(bc2) / bc1
    for start, numel, wd in segments:
        sl = slice(start, start + numel)
        gg = g[sl]
        m, v, n, p = exp_avg[sl], exp_avg_sq[sl], exp_avg_lr[sl], master[sl]
        m.mul_(beta1).add_(gg, alpha=1.0 - beta1)
        v.mul_(beta2).addcmul_(gg, gg, value=1.0 - beta2)
        denom = v.sqrt().add_(eps)
        if wd != 0.0:
            p.add_(p, alpha=-wd * lr)
        ss = torch.full_like(denom, base).div_(denom)
        n.mul_(beta3).add_(ss, alpha=1.0 - beta3)
        ss = torch.minimum(ss, n).mul_(m)
        p.add_(-ss)
    if compute is not None and compute.data_ptr() != master.data_ptr():
        for start, numel, _ in segments:
            compute[start:start + numel].copy_(master[start:start + numel])
