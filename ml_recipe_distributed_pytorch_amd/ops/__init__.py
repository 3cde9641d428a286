"""Fused-op API used by the model.  Dispatch is by device, not by a backend registry:

* CUDA (ROCm/HIP) tensors → hand-written gfx950 kernels in ``_hq_kernels.so`` (fail loudly if absent):
  embedding, LayerNorm, attention, optimizer, heads, and the MFMA GEMMs (``gemm.hip`` NT with fused
  epilogues for every encoder projection forward and dgrad, ``gemm_tn.hip`` split-K weight gradients).
  No vendor BLAS: an untileable shape raises.
* CPU tensors → ``ops.reference`` (pure PyTorch, fp32), which is also the numerics oracle.
* fp32 GPU tensors (``--precision fp32``, the reference's Apex-off mode) → ``ops.f32``: every GEMM-shaped product
  on the own exact-f32 MFMA kernel (``gemm_f32.hip``), the row-wise / elementwise parts and the flash attention on
  the own fp32 kernels (``f32_ops.hip``).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import f32
from . import reference as ref
from . import rng  # noqa: F401
from .._native import kernels


def _k():
    return kernels()


# ------------------------------------------------------------------------------------ embedding
def _hip(t) -> bool:
    """The bf16 / fp8 fused-kernel path handles this GPU tensor (fp32 GPU tensors take ``ops.f32``)."""
    return t.is_cuda and t.dtype != torch.float32


def embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid, out_dtype):
    if _hip(w_word):
        return tuple(_k().embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta,
                                    float(eps), float(p), int(seed), int(opid)))
    if f32.active(w_word):
        return f32.embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid)
    return ref.embed_fwd(ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, beta, eps, p, seed, opid, out_dtype)


def embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
              g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word=-1, pad_pos=-1, seq_len=0):
    """``seq_len`` = L of the [B, L] token layout (0: unknown) — lets the kernel walk one position across
    the batch and sum the position-embedding gradient in registers."""
    if _hip(dy):
        return _k().embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, float(p),
                              int(seed), int(opid), g_word, g_pos, g_type, g_gamma, g_beta, bool(accumulate),
                              int(pad_word), int(pad_pos), int(seq_len))
    if f32.active(dy):
        return f32.embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
                             g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word, pad_pos)
    return ref.embed_bwd(dy, ids, pos_ids, type_ids, w_word, w_pos, w_type, gamma, mean, rstd, p, seed, opid,
                         g_word, g_pos, g_type, g_gamma, g_beta, accumulate, pad_word, pad_pos)


# ------------------------------------------------------------------ residual + dropout + LayerNorm
def _z_or_none(out):
    """ln_fwd's z slot: None when the kernel did not store it (store_z=False)."""
    out = list(out)
    if out[1] is not None and out[1].numel() == 0:
        out[1] = None
    return tuple(out)


def ln_fwd(a, resid, gamma, beta, eps, p, seed, opid, store_z: bool = True):
    """(y, z, mean, rstd).  ``store_z=False`` (GPU): z is not written and comes back None — the backward then
    recomputes x̂ from y (``ln_bwd(..., beta=β)`` with y in z's place), one 2-byte/element store less."""
    if _hip(a):
        return _z_or_none(_k().ln_fwd(a, resid, gamma, beta, float(eps), float(p), int(seed), int(opid),
                                      store_z=bool(store_z)))
    if f32.active(a):
        return f32.ln_fwd(a, resid, gamma, beta, eps, p, seed, opid)
    return ref.ln_fwd(a, resid, gamma, beta, eps, p, seed, opid)


def ln_fwd_q8(a, resid, gamma, beta, eps, p, seed, opid, state: "Fp8DelayedState", store_z: bool = True):
    """``ln_fwd`` that also writes y in e4m3 under ``state`` — the delayed-scaling state of the fp8 GEMM
    that consumes y — so that GEMM needs no separate quantisation pass: (y, z, mean, rstd, y8)."""
    return _z_or_none(_k().ln_fwd(a, resid, gamma, beta, float(eps), float(p), int(seed), int(opid), q8=state.buf,
                                  phase=state.next_phase(), store_z=bool(store_z)))


def ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate, beta=None):
    """(dz, da).  ``beta`` given: ``z`` is the forward output y and x̂ = (y − β)/γ."""
    if _hip(dy):
        return tuple(_k().ln_bwd(dy, dy2, z, gamma, mean, rstd, float(p), int(seed), int(opid),
                                 g_gamma, g_beta, g_bias, bool(accumulate), beta=beta))
    if f32.active(dy):
        return f32.ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate, beta=beta)
    return ref.ln_bwd(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate, beta=beta)


def ln_bwd_q8(dy, dy2, z, gamma, mean, rstd, p, seed, opid, g_gamma, g_beta, g_bias, accumulate,
              state: "Fp8DelayedState", need_da: bool = True, beta=None):
    """``ln_bwd`` that also writes da in e5m2 under ``state`` — the delayed-scaling state of the fp8 dgrad
    GEMM that consumes da: (dz, da, da8); ``need_da=False`` (every consumer reads da8) skips the bf16 da
    (returned as None)."""
    dz, da, da8 = _k().ln_bwd(dy, dy2, z, gamma, mean, rstd, float(p), int(seed), int(opid), g_gamma, g_beta, g_bias,
                              bool(accumulate), q8=state.buf, phase=state.next_phase(), write_da=bool(need_da),
                              beta=beta)
    return dz, (da if need_da else None), da8


# ------------------------------------------------------------------------------------------ GELU
def gelu_fwd(pre):
    if _hip(pre):
        return _k().gelu_fwd(pre)
    if f32.active(pre):
        return _k().f32_gelu_fwd(pre.contiguous())
    return ref.gelu_fwd(pre)


def gelu_bwd(dout, pre, g_bias, accumulate):
    if _hip(dout):
        return _k().gelu_bwd(dout, pre, g_bias, bool(accumulate))
    if f32.active(dout):
        return _k().f32_gelu_bwd(dout.contiguous(), pre.contiguous(), g_bias, bool(accumulate))
    return ref.gelu_bwd(dout, pre, g_bias, accumulate)


# ------------------------------------------------------------------------------------- attention
def attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale):
    """Returns (ctx [T,H], lse [B,nh,L] fp32, keep-bits or None).  The HIP forward stores the dropout
    keep-bits it drew so the backward never re-hashes; the CPU reference regenerates them."""
    if f32.active(qkv):
        ctx, lse = f32.attn_fwd(qkv, key_bias, B, L, nh, p, seed, opid, scale)
        return ctx, lse, None
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


def attn_bwd_q8(dctx, qkv, ctx, lse, key_bias, bits, B, L, nh, p, scale, state: "Fp8DelayedState",
                need_bf16: bool = True):
    """``attn_bwd`` that also writes dQKV in e5m2 under ``state`` — the delayed-scaling state of the fp8 QKV
    dgrad that consumes it: (dqkv, dqkv8, None).  ``need_bf16=False`` (the QKV dgrad and weight gradient
    both read dqkv8): (None, dqkv8, bpart) — no bf16 dQKV; bpart holds column partials of the QKV bias
    gradient (``colsum_into``)."""
    r = _k().attn_bwd_q8(dctx, qkv, ctx, lse, key_bias, bits, int(B), int(L), int(nh), float(p), float(scale),
                         deterministic(), state.buf, state.next_phase(), bool(need_bf16))
    return (r[0], r[1], None) if need_bf16 else (None, r[1], r[2])


def attn_bwd(dctx, qkv, ctx, lse, key_bias, bits, B, L, nh, p, seed, opid, scale):
    if f32.active(dctx):
        return f32.attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale)
    if dctx.is_cuda:
        return _k().attn_bwd(dctx, qkv, ctx, lse, key_bias, bits, int(B), int(L), int(nh), float(p), float(scale),
                             deterministic())
    return ref.attn_bwd(dctx, qkv, ctx, lse, key_bias, B, L, nh, p, seed, opid, scale)


# --------------------------------------------------------------------------------------- linear
# Every projection GEMM on the GPU runs on the hand-written gfx950 MFMA kernels: ``gemm.hip`` (NT, C = A·Bᵀ
# with fused epilogues, every forward projection and dgrad) and ``gemm_tn.hip`` (split-K weight gradients).
# There is no vendor-BLAS fallback: a shape the kernels do not tile raises instead of silently running
# something else (BERT / RoBERTa base and large, and the tiny test config, all tile).
_EPI_NONE, _EPI_BIAS, _EPI_GELU, _EPI_DGELU, _EPI_RESID, _EPI_GELUD, _EPI_DMUL, _EPI_BDR = range(8)
# LN_FUSE: the out-projection / FFN2 GEMM writes z = dropout(x·Wᵀ + b) + resid itself (EPI_BDR) and the
# LayerNorm that follows reads z alone — one HBM pass over [T, H] less per LayerNorm, bitwise the same
# result.  Off by default: the epilogue's residual read and dropout hash are serial with the persistent GEMM's
# MFMA work and cost what the LayerNorm saves (same-box step A/B 3847 vs 3839 samples/s, profiles/r2_ln_fuse)
LN_FUSE = False   # module attribute (tests/test_ln_fuse_gpu.py toggles it); no environment knob
# The encoder LayerNorms' forward skips storing z (151 MB per LayerNorm at B = 256, L = 384) and the backward
# recomputes x̂ = (y − β)/γ from the output y, which the next sublayer keeps anyway (the "memory-efficient"
# LayerNorm backward).  HQ_LN_FROM_Y=0 keeps z (x̂ = (z − mean)·rstd, the exact-input form).
LN_FROM_Y = os.environ.get("HQ_LN_FROM_Y", "1") == "1"


def _check_nt(M: int, N: int, K: int, what: str):
    """Raise unless C[M, N] = A[M, K]·B[N, K]ᵀ tiles on gemm.hip (N % 128 == 0, K % 64 == 0; any M)."""
    if _k().gemm_nt_supported(int(M), int(N), int(K)) <= 0:
        raise RuntimeError(f"{what}: GEMM M={M} N={N} K={K} does not tile on the gfx950 MFMA kernels "
                           "(needs N % 128 == 0 and K % 64 == 0)")


def _bias32(b, b32):
    return b32 if b32 is not None else b.float().contiguous()


def _part(M: int, N: int, K: int, device):
    """Column-partial buffer of a DGELU / DMUL GEMM (one row per M-block of the kernel that runs)."""
    return torch.empty(_k().gemm_nt_part_rows(int(M), int(N), int(K)), N, dtype=torch.float32, device=device)


def linear_fwd(x, w, b, b32=None, kind: str = "plain"):
    """y = x·Wᵀ + b (MFMA NT kernel with the fp32 bias ``b32`` in its epilogue on the GPU)."""
    if f32.active(x):
        return f32.linear_fwd(x, w, b)
    if x.is_cuda:
        _check_nt(x.shape[0], w.shape[0], x.shape[1], f"linear_fwd[{kind}]")
        return _k().gemm_nt(x, w, _EPI_BIAS, bias=_bias32(b, b32))
    return ref.linear_fwd(x, w, b)


def linear_bdr_ln_fwd(x, w, b, b32, resid, kind, gamma, beta, eps, p, seed, opid, store_z: bool = True):
    """LayerNorm(dropout_p(x·Wᵀ + b) + resid) -> (y, z, mean, rstd), bitwise what ``linear_fwd`` followed by
    ``ln_fwd`` computes.  On the GPU with ``LN_FUSE`` the GEMM's EPI_BDR epilogue adds the dropped-out
    projection to the residual and stores z, and the LayerNorm reads z alone (``ln_fwd`` with resid=None);
    otherwise the two ops run as before."""
    if _hip(x) and LN_FUSE and x.shape[0] * w.shape[0] < 2 ** 32:
        _check_nt(x.shape[0], w.shape[0], x.shape[1], f"linear_bdr_ln_fwd[{kind}]")
        z = _k().gemm_nt(x, w, _EPI_BDR, bias=_bias32(b, b32), resid=resid, p=float(p), seed=int(seed), opid=int(opid))
        return tuple(_k().ln_fwd(z, None, gamma, beta, float(eps), 0.0, 0, 0))
    return ln_fwd(linear_fwd(x, w, b, b32, kind), resid, gamma, beta, eps, p, seed, opid, store_z=store_z)


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
    quantiser nor the GEMM ever synchronises with the host.  Forward inputs are e4m3 (scale = 2·amax/448);
    backward activation gradients are e5m2 (scale = 64·amax/57344, ``grad=True``; hq_common.h margins)."""

    def __init__(self, device, buf: Optional[torch.Tensor] = None, grad: bool = False):
        self.buf = torch.zeros(4, dtype=torch.float32, device=device) if buf is None else buf
        self.step = 0
        self.grad = grad

    @property
    def calibrated(self) -> bool:
        """True once a previous production recorded an amax, i.e. the scale in use now is derived from
        real data (a gradient state has no current-scaling seed: its consumer runs in bf16 until then)."""
        return self.step >= 2

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


def gelud_code():
    """(lo, step) of the fp8 path's 8-bit gelu' code (hq_kernels.h kHqGdLo / kHqGdStep): g ≈ lo + q·step."""
    return _k().gelud_code()


def gelud_encode(g: torch.Tensor) -> torch.Tensor:
    """gelu' → the 8-bit code, as the fp8 FFN1 epilogue writes it (hq_gd_encode8: ONE fp32 fma g·inv + off with
    inv = 1/step, off = −lo/step, round to nearest even, clamp 0…255).  On the GPU this is the device encoder
    itself (``gelud_encode8`` kernel), so both paths write identical bytes; the host form mirrors it with the
    constants taken from ``gelud_code()``."""
    if g.is_cuda:
        return _k().gelud_encode8(g.to(torch.bfloat16).contiguous())
    inv, off = _k().gelud_code_enc()
    inv = torch.tensor(inv, dtype=torch.float32)
    off = torch.tensor(off, dtype=torch.float32)
    q = torch.round(torch.addcmul(off.expand(g.shape), g.float(), inv.expand(g.shape)))
    return q.clamp_(0, 255).to(torch.uint8)


def gelud_decode(q: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    lo, step = gelud_code()
    return (q.float() * step + lo).to(dtype)


def linear_gelu_fwd_fp8(x, w8s, b32, in_state: Fp8DelayedState, out_state: Fp8DelayedState, x8=None,
                        need_act: bool = True):
    """FFN1 in fp8 on the own block-scaled MFMA kernel (gemm_fp8.hip): returns (gelu'(pre), act, act8) — act in
    bf16 and in e4m3 under ``out_state``'s delayed scale for the FFN2 fp8 GEMM; None when the shape does not tile
    (caller falls back).  ``need_act=False`` (the caller knows the backward will run the FFN2 dgrad and weight
    gradient in fp8) skips the bf16 act (returned as None) and stores gelu' as the 8-bit code of ``gelud_code()``
    that the fp8 dgrad reads; otherwise gelu' is stored in bf16 for the bf16 dgrad (no code, no decode error).
    ``x8``: the input already in e4m3 under ``in_state`` (LN forward's fp8 output), else it is quantised here."""
    M, K, N = x.shape[0], x.shape[1], w8s[0].shape[0]
    if not _k().gemm_fp8_supported(M, N, K):
        return None
    if x8 is None:
        x8 = in_state.quantize(x)
    w8, sw = w8s
    gd = torch.empty(M, N, dtype=torch.bfloat16 if need_act else torch.uint8, device=x.device)
    act8 = torch.empty(M, N, dtype=torch.float8_e4m3fn, device=x.device)
    act = _k().gemm_fp8(x8, w8, _EPI_GELUD, b32, in_state.scale, sw.reshape(1).float(), pre=gd, out8=act8,
                        state=out_state.buf, phase=out_state.next_phase(), write_out=bool(need_act))
    return gd, (act if need_act else None), act8


def linear_dgrad_fp8(dy8, dy_state: Fp8DelayedState, wt8s):
    """dy·W for an e5m2 gradient ``dy8`` written by its producer under ``dy_state``, on the fp8 MFMA kernel
    (gemm_fp8.hip EPI_NONE) against the e4m3 Wᵀ copy ``wt8s`` = (Wᵀ fp8 [in, out], dequant scale) from
    ParamStore.view_fp8_t; bf16 out."""
    wt8, sw = wt8s
    return _k().gemm_fp8(dy8, wt8, _EPI_NONE, None, dy_state.scale, sw.reshape(1).float())


def linear_dgrad_add_fp8(dy8, dy_state: Fp8DelayedState, wt8s, resid):
    """resid + dy·W for an e5m2 gradient (the QKV dgrad plus the residual-gradient add, gemm_fp8.hip
    EPI_RESID) against the e4m3 Wᵀ copy; bf16 out."""
    wt8, sw = wt8s
    return _k().gemm_fp8(dy8, wt8, _EPI_RESID, None, dy_state.scale, sw.reshape(1).float(), resid=resid)


def linear_dgrad_gelu_fp8(dy8, dy_state: Fp8DelayedState, wt8s, gd, g_bias, accumulate, out_state: Fp8DelayedState,
                          need_bf16: bool = True):
    """FFN2 dgrad in fp8: dpre = (dy·W) ⊙ gelu'(pre) (``gd``: the gelu' code stored by the fp8 forward; a bf16
    gelu' from a bf16 forward is encoded first), the FFN1 bias gradient from the epilogue's column sums, and dpre
    also in e5m2 under ``out_state`` for the FFN1 dgrad: (dpre, dpre8); ``need_bf16=False`` (every consumer reads
    dpre8) skips the bf16 dpre (returned as None)."""
    wt8, sw = wt8s
    if gd.dtype != torch.uint8:
        gd = gelud_encode(gd)
    M, N = dy8.shape[0], wt8.shape[0]
    part = torch.empty(M // 256, N, dtype=torch.float32, device=dy8.device)
    dpre8 = torch.empty(M, N, dtype=torch.float8_e5m2, device=dy8.device)
    dpre = _k().gemm_fp8(dy8, wt8, _EPI_DMUL, None, dy_state.scale, sw.reshape(1).float(), pre=gd, out8=dpre8,
                         state=out_state.buf, phase=out_state.next_phase(), part=part, write_out=bool(need_bf16))
    if g_bias is not None:
        _k().colsum_into(part, g_bias, bool(accumulate))
    return (dpre if need_bf16 else None), dpre8


def fp8_wgrad_ok(T: int, N: int, K: int) -> bool:
    return _k().gemm_tn8_splits(int(T), int(N), int(K)) > 0


def linear_wgrad_fp8(dy8, dy_state: Fp8DelayedState, x8, x_state: Fp8DelayedState, g_w, accumulate):
    """g_w (fp32 arena view) (+)= dyᵀ·x from the e5m2 gradient and the e4m3 forward input their producers
    wrote (gemm_tn.hip gemm_tn8_kernel, split-K, dequantised by both states' scales).  No bias: the fp8 step
    takes its bias gradients from the LayerNorm backward / DMUL column sums (QKV's wgrad stays bf16)."""
    _k().gemm_tn8(dy8, x8, dy_state.scale, x_state.scale, g_w, bool(accumulate))


def linear_gelu_fwd(x, w, b, b32=None):
    """(pre, act) with pre = x·Wᵀ + b, act = gelu(pre) — the CPU oracle form; the GPU uses
    ``linear_gelu_fwd_d`` (derivative stored instead of pre)."""
    if _hip(x):
        _check_nt(x.shape[0], w.shape[0], x.shape[1], "linear_gelu_fwd")
        pre = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        act = _k().gemm_nt(x, w, _EPI_GELU, bias=_bias32(b, b32), pre=pre)
        return pre, act
    pre = f32.linear_fwd(x, w, b) if f32.active(x) else ref.linear_fwd(x, w, b)
    return pre, gelu_fwd(pre)


def linear_gelu_fwd_d(x, w, b, b32=None):
    """(saved, act, is_deriv).  GPU: one MFMA GEMM whose epilogue evaluates Φ and φ once and stores
    gelu'(pre) (bf16) beside act, so the backward needs one multiply per element (``linear_dgrad_gelu_d``);
    CPU / fp32 GPU: (pre, act, False)."""
    if _hip(x):
        _check_nt(x.shape[0], w.shape[0], x.shape[1], "linear_gelu_fwd_d")
        gd = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device)
        act = _k().gemm_nt(x, w, _EPI_GELUD, bias=_bias32(b, b32), pre=gd)
        return gd, act, True
    pre, act = linear_gelu_fwd(x, w, b, b32)
    return pre, act, False


def linear_dgrad_gelu_d(dy, w, saved, is_deriv, g_bias, accumulate, wt=None):
    """Backward of ``linear_gelu_fwd_d``: dpre = (dy·W) ⊙ gelu'(pre) with the FFN1 bias gradient."""
    if not is_deriv:
        return linear_dgrad_gelu(dy, w, saved, g_bias, accumulate, wt)
    M, N = dy.shape[0], w.shape[1]
    assert wt is not None, "stored-derivative GELU backward needs the Wᵀ working copy"
    _check_nt(M, N, dy.shape[1], "linear_dgrad_gelu_d")
    if saved.dtype == torch.uint8:   # the fp8 forward's gelu' code (written only when the fp8 dgrad was expected)
        saved = gelud_decode(saved)
    part = _part(M, N, dy.shape[1], dy.device)
    dpre = _k().gemm_nt(dy, wt, _EPI_DMUL, pre=saved, part=part)
    if g_bias is not None:
        _k().colsum_into(part, g_bias, bool(accumulate))
    return dpre


def linear_dgrad(dy, w, wt=None):
    """dy·W.  GPU: NT kernel on the Wᵀ working copy ``wt`` (ParamStore.view_t)."""
    if f32.active(dy):
        return f32.linear_dgrad(dy, w)
    if dy.is_cuda:
        assert wt is not None, "GPU dgrad needs the Wᵀ working copy"
        _check_nt(dy.shape[0], w.shape[1], dy.shape[1], "linear_dgrad")
        return _k().gemm_nt(dy, wt, _EPI_NONE)
    return ref.linear_dgrad(dy, w)


def linear_dgrad_add(dy, w, resid, wt=None):
    """resid + dy·W (fuses the residual-gradient add)."""
    if f32.active(dy):
        return f32.linear_dgrad(dy, w, resid)
    if dy.is_cuda:
        assert wt is not None, "GPU dgrad needs the Wᵀ working copy"
        _check_nt(dy.shape[0], w.shape[1], dy.shape[1], "linear_dgrad_add")
        return _k().gemm_nt(dy, wt, _EPI_RESID, resid=resid)
    return ref.linear_dgrad_add(dy, w, resid)


def linear_dgrad_gelu(dy, w, pre, g_bias, accumulate, wt=None):
    """dpre = (dy·W) ⊙ gelu'(pre) and g_bias (+)= Σ_rows dpre — the dgrad of the layer after GELU
    fused with the GELU backward and the bias gradient of the layer before it."""
    if f32.active(dy):
        return gelu_bwd(f32.linear_dgrad(dy, w), pre, g_bias, accumulate)
    if dy.is_cuda:
        assert wt is not None, "GPU dgrad needs the Wᵀ working copy"
        M, N = dy.shape[0], w.shape[1]
        _check_nt(M, N, dy.shape[1], "linear_dgrad_gelu")
        part = _part(M, N, dy.shape[1], dy.device)
        dpre = _k().gemm_nt(dy, wt, _EPI_DGELU, pre=pre, part=part)
        if g_bias is not None:
            _k().colsum_into(part, g_bias, bool(accumulate))
        return dpre
    return gelu_bwd(ref.linear_dgrad(dy, w), pre, g_bias, accumulate)


def linear_wgrad(dy, x, g_w, g_b, accumulate):
    """g_w (fp32 arena view) (+)= dyᵀ·x with fp32 GEMM output; g_b (+)= column sums of dy.
    GPU: the split-K TN MFMA kernel (gemm_tn.hip) with the bias gradient fused; raises for shapes it does
    not tile (N, K multiples of 128)."""
    if f32.active(dy):
        return f32.linear_wgrad(dy, x, g_w, g_b, accumulate)
    if dy.is_cuda:
        T, N = dy.shape
        K = x.shape[1]
        if not g_w.is_contiguous() or _k().gemm_tn_splits(T, N, K) <= 0:
            raise RuntimeError(f"linear_wgrad: dW[{N}, {K}] over T={T} tokens does not tile on gemm_tn "
                               "(needs N % 128 == 0, K % 128 == 0 and a contiguous fp32 gradient view)")
        fuse_b = g_b is not None and g_b.is_contiguous()
        _k().gemm_tn(dy, x, g_w, bool(accumulate), 0, g_b if fuse_b else None)
        if g_b is not None and not fuse_b:
            _k().bias_grad(dy, g_b, bool(accumulate))
        return
    ref.linear_wgrad(dy, x, g_w, g_b, accumulate)


def colsum_into(part, out, accumulate):
    """out (+)= Σ_rows part (fp32 column partials, e.g. the QKV bias gradient of the fp8 backward)."""
    _k().colsum_into(part, out, bool(accumulate))


def bias_grad(dy, g_b, accumulate):
    if _hip(dy):
        return _k().bias_grad(dy, g_b, bool(accumulate))
    ref._acc(g_b, dy.float().sum(0), accumulate)
