"""Fused-op API used by the model.  Dispatch is by device, not by a backend registry:

* CUDA (ROCm/HIP) tensors → hand-written gfx950 kernels in ``_hq_kernels.so`` (fail loudly if absent):
  embedding, LayerNorm, attention, optimizer, and the MFMA GEMMs (``gemm.hip`` NT with fused epilogues
  for every encoder projection forward and dgrad, ``gemm_tn.hip`` split-K weight gradients).  hipBLASLt
  (``torch.addmm/mm``) is only the fallback for shapes the MFMA kernels do not tile (see ``_mfma``) and
  for the tiny pooler / QA-head GEMMs.
* CPU tensors → ``ops.reference`` (pure PyTorch, fp32), which is also the numerics oracle.
"""
from __future__ import annotations

import os
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
              g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word=-1, pad_pos=-1, seq_len=0):
    """``seq_len`` = L of the [B, L] token layout (0: unknown) — lets the kernel walk one position across
    the batch and sum the position-embedding gradient in registers."""
    if dy.is_cuda:
        return _k().embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, float(p),
                              int(seed), int(opid), g_word, g_pos, g_type, g_gamma, g_beta, bool(accumulate),
                              int(pad_word), int(pad_pos), int(seq_len))
    return ref.embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
                         g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word, pad_pos)


# ------------------------------------------------------------------ residual + dropout + LayerNorm
def ln_fwd(a, resid, gamma, beta, eps, p, seed, opid):
    if a.is_cuda:
        return tuple(_k().ln_fwd(a, resid, gamma, beta, float(eps), float(p), int(seed), int(opid)))
    return ref.ln_fwd(a, resid, gamma, beta, eps, p, seed, opid)


def ln_fwd_q8(a, resid, gamma, beta, eps, p, seed, opid, state: "Fp8DelayedState"):
    """``ln_fwd`` that also writes y in e4m3 under ``state`` — the delayed-scaling state of the fp8 GEMM
    that consumes y — so that GEMM needs no separate quantisation pass: (y, z, mean, rstd, y8)."""
    return tuple(_k().ln_fwd(a, resid, gamma, beta, float(eps), float(p), int(seed), int(opid), q8=state.buf,
                             phase=state.next_phase()))


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
    """Returns (ctx [T,H], lse [B,nh,L] fp32, keep-bits or None).  The HIP forward stores the dropout
    keep-bits it drew so the backward never re-hashes; the CPU reference regenerates them."""
    if qkv.is_cuda:
        ctx, lse, bits = _k().attn_fwd(qkv, key_bias, int(B), int(L), int(nh), float(p), int(seed), int(opid),
                                       float(scale))
        return ctx, lse, bits
    ctx, lse = ref.attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale)
    return ctx, lse, None


def deterministic() -> bool:
    """Bitwise run-to-run reproducible kernels wanted: ``torch.use_deterministic_algorithms(True)`` or
    ``HQ_DETERMINISTIC=1``.  Only the attention backward has a faster order-nondeterministic path (the
    single-kernel backward sums dQ over key slices with LDS float atomics); the embedding-gradient
    scatter stays atomic either way."""
    return torch.are_deterministic_algorithms_enabled() or os.environ.get("HQ_DETERMINISTIC", "0") == "1"


def attn_fwd_q8(qkv, key_bias, B, L, nh, p, seed, opid, scale, state: "Fp8DelayedState"):
    """``attn_fwd`` that also writes ctx in e4m3 under ``state`` — the delayed-scaling state of the
    out-projection that consumes it (producer-side quantisation): (ctx, lse, keep-bits, ctx8)."""
    ctx, lse, bits, ctx8 = _k().attn_fwd(qkv, key_bias, int(B), int(L), int(nh), float(p), int(seed), int(opid),
                                         float(scale), q8=state.buf, phase=state.next_phase())
    return ctx, lse, bits, ctx8


def attn_bwd(dctx, qkv, ctx, lse, key_bias, bits, B, L, nh, p, seed, opid, scale):
    if dctx.is_cuda:
        return _k().attn_bwd(dctx, qkv, ctx, lse, key_bias, bits, int(B), int(L), int(nh), float(p), float(scale),
                             deterministic())
    return ref.attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale)


# --------------------------------------------------------------------------------------- linear
# Which projection GEMMs run on the hand-written MFMA NT kernel (gemm.hip) instead of hipBLASLt.
#   HQ_GEMM=auto (default): the GEMMs whose epilogue fuses an elementwise pass — FFN1 + GELU,
#     FFN2-dgrad + dGELU + FFN1 bias-grad (1.08x / 1.40x vs hipBLASLt + separate kernel at b256,
#     profiles/) and the QKV dgrad + residual-gradient add (torch.addmm first copies the residual
#     into the output: +56 µs at b256), plus the plain dgrads, for every M (gemm.hip picks 256-row or
#     128² tiles by M alignment and CU fill).  Weight gradients take the split-K TN kernel (gemm_tn.hip).
#     Plain forward projections follow FWD_MFMA below (all three on the MFMA kernel by default);
#   HQ_GEMM=mfma: every supported shape;  HQ_GEMM=blas: none.
_EPI_NONE, _EPI_BIAS, _EPI_GELU, _EPI_DGELU, _EPI_RESID, _EPI_GELUD, _EPI_DMUL, _EPI_BDR = range(8)
_GEMM_MODE = os.environ.get("HQ_GEMM", "auto").lower()
# Plain forward projections (bias epilogue) that take the MFMA kernel in auto mode, by name: qkv | out | ffn2.
# In the full b256 step hipBLASLt's QKV pick runs 381 µs vs 316 µs standalone while the MFMA kernel holds
# ~337 µs (+0.4 % step); the out-projection / FFN2 forwards are step-neutral either way (profiles/s3_ab), so
# all three default to the own kernel and the bf16 encoder runs no vendor GEMM (the tiny pooler/head
# GEMMs stay in torch).
FWD_MFMA = {k for k in os.environ.get("HQ_FWD_MFMA", "qkv,out,ffn2").split(",") if k}
GELU_DERIV = os.environ.get("HQ_GELU_DERIV", "1") == "1"   # FFN1 stores gelu'(pre) (linear_gelu_fwd_d)
# HQ_LN_FUSE=1: the out-projection / FFN2 GEMM writes z = dropout(x·Wᵀ + b) + resid itself (EPI_BDR) and the
# LayerNorm that follows reads z alone — one HBM pass over [T, H] less per LayerNorm, bitwise the same
# result.  Off by default: the epilogue's residual read and dropout hash are serial with the persistent GEMM's
# MFMA work and cost what the LayerNorm saves (same-box step A/B 3847 vs 3839 samples/s, profiles/r2_ln_fuse)
LN_FUSE = os.environ.get("HQ_LN_FUSE", "0") == "1"


def set_gemm_mode(mode: str) -> str:
    """Switch the projection-GEMM policy at runtime (auto | mfma | blas); returns the previous mode."""
    global _GEMM_MODE
    prev, _GEMM_MODE = _GEMM_MODE, mode.lower()
    return prev


def _mfma(M: int, N: int, K: int, kind: str = "plain") -> bool:
    """Every projection shape with N % 128 == 0 and K % 64 == 0 runs on the own MFMA kernels: the
    256-row kernels where M % 256 == 0 and the grid fills the CUs, the 128²-tile kernel otherwise
    (M tails of dynamically padded batches, small micro-batches, low-fill grids) — gemm.hip picks."""
    if _GEMM_MODE == "blas":
        return False
    if _k().gemm_nt_supported(int(M), int(N), int(K)) <= 0:
        return False
    if _GEMM_MODE == "mfma":
        return True
    return kind in ("dgelu", "gelu", "resid", "dgrad") or kind in FWD_MFMA


def _part(M: int, N: int, K: int, device):
    """Column-partial buffer of a DGELU / DMUL GEMM (one row per M-block of the kernel that runs)."""
    return torch.empty(_k().gemm_nt_part_rows(int(M), int(N), int(K)), N, dtype=torch.float32, device=device)


def linear_fwd(x, w, b, b32=None, kind: str = "plain"):
    """y = x·Wᵀ + b.  GPU: hipBLASLt (bias epilogue) or the MFMA NT kernel (fp32 ``b32`` bias); ``kind``
    names the projection (qkv | out | ffn2) for the FWD_MFMA policy."""
    if x.is_cuda:
        if b32 is not None and _mfma(x.shape[0], w.shape[0], x.shape[1], kind):
            return _k().gemm_nt(x, w, _EPI_BIAS, bias=b32)
        return torch.addmm(b, x, w.t()) if b is not None else torch.mm(x, w.t())
    return ref.linear_fwd(x, w, b)


def linear_bdr_ln_fwd(x, w, b, b32, resid, kind, gamma, beta, eps, p, seed, opid):
    """LayerNorm(dropout_p(x·Wᵀ + b) + resid) -> (y, z, mean, rstd), bitwise what ``linear_fwd`` followed by
    ``ln_fwd`` computes.  On the GPU with the own MFMA kernel the GEMM's EPI_BDR epilogue adds the dropped-out
    projection to the residual and stores z, and the LayerNorm reads z alone (``ln_fwd`` with resid=None);
    otherwise the two ops run as before."""
    if (x.is_cuda and LN_FUSE and b32 is not None and _mfma(x.shape[0], w.shape[0], x.shape[1], kind)
            and x.shape[0] * w.shape[0] < 2 ** 32):
        z = _k().gemm_nt(x, w, _EPI_BDR, bias=b32, resid=resid, p=float(p), seed=int(seed), opid=int(opid))
        return tuple(_k().ln_fwd(z, None, gamma, beta, float(eps), 0.0, 0, 0))
    return ln_fwd(linear_fwd(x, w, b, b32, kind), resid, gamma, beta, eps, p, seed, opid)


def linear_fwd_fp8(x, w8s, b):
    """y = x·Wᵀ + b with both operands in OCP fp8 e4m3 (x under per-tensor current scaling, one amax pass +
    one quantisation pass) on the own fp8 MFMA kernel (gemm_fp8.hip), bf16 out.  ``w8s`` = (W fp8 [N,K],
    dequant scale) from ParamStore.view_fp8.  The training step uses the producer-quantised form
    (``linear_fwd_fp8_own``); this is the standalone op."""
    x8, sx = _k().fp8_quantize(x)
    w8, sw = w8s
    return _k().gemm_fp8(x8, w8, _EPI_BIAS, b.float().contiguous(), sx.reshape(1).float(), sw.reshape(1).float())


class Fp8DelayedState:
    """Per-site delayed-scaling state of an fp8 GEMM input: a device f32[4] (three rotating amax slots
    + the scale in use, see gemm_fp8.hip) and a host step counter selecting the slots — so neither the
    quantiser nor the GEMM ever synchronises with the host."""

    def __init__(self, device, buf: Optional[torch.Tensor] = None):
        self.buf = torch.zeros(4, dtype=torch.float32, device=device) if buf is None else buf
        self.step = 0

    def next_phase(self) -> int:
        ph = self.step % 3
        self.step += 1
        return ph

    @property
    def scale(self):  # dequant scale of the most recent quantisation (1-element device view)
        return self.buf[3:4]

    def quantize(self, x):
        """x (bf16) -> e4m3 in one pass under the delayed scale; the very first call seeds the
        "previous amax" slot from x itself (current scaling) instead of falling back to a unit scale."""
        ph = self.next_phase()
        if self.step == 1:
            _, s = _k().fp8_quantize(x)           # s = amax / 448 (device scalar)
            self.buf[(ph + 2) % 3] = s * 448.0    # slots hold float bits; amax >= 0 orders as uint
        return _k().fp8_quant_delayed(x, self.buf, ph)


def fp8_gemm_ok(M: int, N: int, K: int) -> bool:
    return bool(_k().gemm_fp8_supported(int(M), int(N), int(K)))


def linear_fwd_fp8_own(x8, x_state: Fp8DelayedState, w8s, b32):
    """y = x8·W8ᵀ·s_x·s_w + b on the own block-scaled fp8 MFMA kernel (gemm_fp8.hip, bias epilogue) for an
    e4m3 input written by its producer under ``x_state`` (LN forward, FFN1 epilogue, or ``quantize``)."""
    w8, sw = w8s
    return _k().gemm_fp8(x8, w8, _EPI_BIAS, b32, x_state.scale, sw.reshape(1).float())


def linear_gelu_fwd_fp8(x, w8s, b32, in_state: Fp8DelayedState, out_state: Fp8DelayedState, x8=None):
    """FFN1 in fp8 on the own block-scaled MFMA kernel (gemm_fp8.hip): returns (gelu'(pre), act, act8)
    — act in bf16 (saved for the FFN2 weight gradient) and in e4m3 under ``out_state``'s delayed scale
    for the FFN2 fp8 GEMM; None when the shape does not tile (caller falls back).  ``x8``: the input
    already in e4m3 under ``in_state`` (LN forward's fp8 output), else it is quantised here."""
    M, K, N = x.shape[0], x.shape[1], w8s[0].shape[0]
    if not _k().gemm_fp8_supported(M, N, K):
        return None
    if x8 is None:
        x8 = in_state.quantize(x)
    w8, sw = w8s
    gd = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    act8 = torch.empty(M, N, dtype=torch.float8_e4m3fn, device=x.device)
    act = _k().gemm_fp8(x8, w8, _EPI_GELUD, b32, in_state.scale, sw.reshape(1).float(), pre=gd, out8=act8,
                        state=out_state.buf, phase=out_state.next_phase())
    return gd, act, act8


def linear_gelu_fwd(x, w, b, b32=None):
    """(pre, act) with pre = x·Wᵀ + b, act = gelu(pre).  GPU: one MFMA GEMM with the GELU epilogue
    (pre stored for the backward) when the shape allows, else GEMM + gelu kernel."""
    if x.is_cuda and b32 is not None and _mfma(x.shape[0], w.shape[0], x.shape[1], "gelu"):
        pre = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        act = _k().gemm_nt(x, w, _EPI_GELU, bias=b32, pre=pre)
        return pre, act
    pre = linear_fwd(x, w, b, b32)
    return pre, gelu_fwd(pre)


def linear_gelu_fwd_d(x, w, b, b32=None):
    """(saved, act, is_deriv): like ``linear_gelu_fwd`` but, on the MFMA path, ``saved`` is gelu'(pre)
    (bf16) instead of pre — the epilogue evaluates Φ and φ anyway, and the backward then needs one
    multiply per element instead of a GELU-derivative evaluation (``linear_dgrad_gelu_d``)."""
    if GELU_DERIV and x.is_cuda and b32 is not None and _mfma(x.shape[0], w.shape[0], x.shape[1], "gelu"):
        gd = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        act = _k().gemm_nt(x, w, _EPI_GELUD, bias=b32, pre=gd)
        return gd, act, True
    pre, act = linear_gelu_fwd(x, w, b, b32)
    return pre, act, False


def linear_dgrad_gelu_d(dy, w, saved, is_deriv, g_bias, accumulate, wt=None):
    """Backward of ``linear_gelu_fwd_d``: dpre = (dy·W) ⊙ gelu'(pre) with the FFN1 bias gradient."""
    if not is_deriv:
        return linear_dgrad_gelu(dy, w, saved, g_bias, accumulate, wt)
    M, N = dy.shape[0], w.shape[1]
    assert wt is not None, "stored-derivative GELU backward needs the MFMA path (Wᵀ working copy)"
    part = _part(M, N, dy.shape[1], dy.device)
    dpre = _k().gemm_nt(dy, wt, _EPI_DMUL, pre=saved, part=part)
    if g_bias is not None:
        _k().colsum_into(part, g_bias, bool(accumulate))
    return dpre


def linear_dgrad(dy, w, wt=None):
    """dy·W.  ``wt`` = Wᵀ working copy (ParamStore.view_t) enables the NT MFMA kernel."""
    if dy.is_cuda:
        if wt is not None and _mfma(dy.shape[0], w.shape[1], dy.shape[1], "dgrad"):
            return _k().gemm_nt(dy, wt, _EPI_NONE)
        return torch.mm(dy, w)
    return ref.linear_dgrad(dy, w)


def linear_dgrad_add(dy, w, resid, wt=None):
    """resid + dy·W (fuses the residual-gradient add)."""
    if dy.is_cuda:
        if wt is not None and _mfma(dy.shape[0], w.shape[1], dy.shape[1], "resid"):
            return _k().gemm_nt(dy, wt, _EPI_RESID, resid=resid)
        return torch.addmm(resid, dy, w)
    return ref.linear_dgrad_add(dy, w, resid)


def linear_dgrad_gelu(dy, w, pre, g_bias, accumulate, wt=None):
    """dpre = (dy·W) ⊙ gelu'(pre) and g_bias (+)= Σ_rows dpre — the dgrad of the layer after GELU
    fused with the GELU backward and the bias gradient of the layer before it."""
    if dy.is_cuda and wt is not None and _mfma(dy.shape[0], w.shape[1], dy.shape[1], "dgelu"):
        M, N = dy.shape[0], w.shape[1]
        part = _part(M, N, dy.shape[1], dy.device)
        dpre = _k().gemm_nt(dy, wt, _EPI_DGELU, pre=pre, part=part)
        if g_bias is not None:
            _k().colsum_into(part, g_bias, bool(accumulate))
        return dpre
    return gelu_bwd(linear_dgrad(dy, w, wt), pre, g_bias, accumulate)


def _wgrad_splits(T: int, N: int, K: int) -> int:
    """Split-K factor for dW = dyᵀ·x (reduction over T tokens, output only N×K): hipBLASLt runs these
    long-K / small-MN GEMMs far below peak (a 768×768 output is 9 tiles of 256² for 256 CUs), so the
    T axis is split into a batched GEMM with fp32 partials.  Factors from the MI355X sweep
    (tools/wgrad_bench.py, profiles/): ~6k tokens per split for >= 32 output tiles, ~3k for 10-31,
    ~1.5k for <= 9, at most 16 splits (T = 98304: 16 everywhere, 430-480 µs → 0.8-1.0 PF)."""
    tiles = max(1, (N * K) // (256 * 256))
    per = 6144 if tiles >= 32 else (3072 if tiles > 9 else 1536)
    target = max(1, min(16, T // per))
    s = 1
    while s * 2 <= target and T % (s * 2) == 0 and T // (s * 2) >= 1024:
        s *= 2
    return s


def linear_wgrad(dy, x, g_w, g_b, accumulate):
    """g_w (fp32 arena view) (+)= dyᵀ·x with fp32 GEMM output; g_b (+)= column sums of dy.
    GPU: the hand-written split-K TN MFMA kernel (gemm_tn.hip; 1.14-1.31x hipBLASLt's batched split-K
    on the BERT shapes, profiles/) whenever the shape tiles (N, K multiples of 256, T of 64);
    hipBLASLt otherwise (``HQ_GEMM=blas`` forces it)."""
    if dy.is_cuda:
        T, N = dy.shape
        K = x.shape[1]
        if _GEMM_MODE != "blas" and g_w.is_contiguous() and _k().gemm_tn_splits(T, N, K) > 0:
            _k().gemm_tn(dy, x, g_w, bool(accumulate), 0, g_b if (g_b is not None and g_b.is_contiguous()) else None)
            if g_b is not None and not g_b.is_contiguous():
                _k().bias_grad(dy, g_b, bool(accumulate))
            return
        s = _wgrad_splits(T, N, K)
        if s > 1:
            part = torch.bmm(dy.view(s, T // s, N).transpose(1, 2), x.view(s, T // s, K), out_dtype=torch.float32)
            if accumulate:
                g_w.add_(part.sum(0))
            else:
                torch.sum(part, 0, out=g_w)
        elif accumulate:
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
