"""Counter-based dropout RNG shared bit-exactly by the CPU reference ops and the HIP kernels.

Dropout masks are never stored: every fused kernel (embedding+LN, residual+LN, attention P)
regenerates its keep-mask from ``(seed, opid, element index)`` in both forward and backward.
A full Philox4x32-10 per element would make the attention forward VALU-bound on CDNA4
(≈100 VALU per 4 draws vs 8 MFMAs per 32×32 tile, see cdna_hip_programming.md §B attention),
so one cheap mixing hash yields TWO 16-bit uniforms.  The per-element hash avoids 32-bit
multiplies (quarter rate on CDNA4) and uses the full-rate 24-bit multiply ``v_mul_u32_u24``:

    key  = fmix32(seed ^ (opid * 0x9E3779B9))                      (host, once per op)
    x    = (idx >> 1) ^ key
    x   ^= x >> 16;  x = (x & 0xFFFFFF) * 0x9E3779;  x ^= x >> 15
    x    = (x & 0xFFFFFF) * 0xC2B2AE;  x ^= x >> 16               (all mod 2^32)
    u16  = (x >> (16 * (idx & 1))) & 0xFFFF

Quality (4M pairs): per-input-bit avalanche 0.4996-0.5003, drop rate 0.10005 at p = 0.1,
|correlation| < 3e-4 between the two halves, neighbouring pairs and a 192-pair stride.
    keep = u16 >= thr,   thr = round(p * 65536),   scale = 65536 / (65536 - thr)

``scale`` makes the masked activation exactly unbiased for the quantised keep probability.
The same formulas live in ``csrc/include/hq_common.h`` (``hq_keep``).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF


def fmix32_int(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def op_key(seed: int, opid: int) -> int:
    return fmix32_int((seed & M32) ^ ((opid * 0x9E3779B9) & M32))


def threshold(p: float) -> int:
    return int(round(float(p) * 65536.0))


def keep_scale(p: float) -> float:
    thr = threshold(p)
    return 65536.0 / (65536.0 - thr) if thr < 65536 else 0.0


def _fmix32_t(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return h


def pair_hash_t(pair: torch.Tensor, key: int) -> torch.Tensor:
    """The per-pair hash of ``hq_pair_hash`` (int64 tensors holding u32 values)."""
    x = pair ^ key
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * 0x9E3779) & M32
    x = x ^ (x >> 15)
    x = ((x & 0xFFFFFF) * 0xC2B2AE) & M32
    return x ^ (x >> 16)


def keep_mask_from_index(idx: torch.Tensor, seed: int, opid: int, p: float) -> torch.Tensor:
    """Keep-mask (bool) for int64 element indices ``idx`` (any shape)."""
    key = op_key(seed, opid)
    h = pair_hash_t(idx >> 1, key)
    u16 = (h >> ((idx & 1) * 16)) & 0xFFFF
    return u16 >= threshold(p)


def keep_mask(shape, seed: int, opid: int, p: float, device=None) -> torch.Tensor:
    numel = 1
    for s in shape:
        numel *= int(s)
    assert numel < (1 << 32), "dropout element index must fit 32 bits"
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    return keep_mask_from_index(idx, seed, opid, p).view(*shape)


def dropout_apply(x: torch.Tensor, seed: int, opid: int, p: float) -> torch.Tensor:
    if p <= 0.0:
        return x
    m = keep_mask(x.shape, seed, opid, p, device=x.device)
    return x * m.to(x.dtype) * keep_scale(p)
