"""Flat parameter / gradient arenas.

All trainable tensors live in three contiguous device buffers:

* ``master``  fp32 — the ``nn.Parameter`` objects are *views* into it (HF names, so
  ``state_dict()`` matches ``transformers.BertModel`` + the reference QA heads);
* ``compute`` bf16 — working copy read by the GEMMs / fused kernels, rewritten by the fused
  optimizer kernel every step (on CPU / fp32 it *is* ``master``);
* ``grad``    fp32 — ``param.grad`` are views; the fused layer backward kernels write weight
  gradients straight into it, so the gradient reducer all-reduces contiguous arena slices
  with no bucket copies (replaces the torch DDP Reducer's copy-in/copy-out).

Arena order = backward-readiness order (QA heads, pooler, layer N-1 … layer 0, embeddings), so
every all-reduce bucket is one contiguous range and buckets complete front to back.
Fused tensors (QKV = query‖key‖value rows) are single arena entries whose HF-named pieces are
row slices; every entry starts 256-byte aligned for 16-B vector access in the kernels.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

_ALIGN = 64  # elements (256 B of fp32, 128 B of bf16)


@dataclass
class Entry:
    key: str
    shape: Tuple[int, ...]
    group: str
    init: str = "normal"                      # normal | zeros | ones
    views: List[Tuple[str, int, int]] = field(default_factory=list)   # (hf_name, row0, row1)
    offset: int = 0

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


def no_decay(name: str) -> bool:
    """Reference ``init.py:125-129``: no weight decay for bias / LayerNorm params."""
    return any(nd in name for nd in ("bias", "LayerNorm.bias", "LayerNorm.weight"))


class ParamStore:
    def __init__(self, entries: Sequence[Entry]):
        self.entries: List[Entry] = list(entries)
        off = 0
        for e in self.entries:
            off = (off + _ALIGN - 1) // _ALIGN * _ALIGN
            e.offset = off
            off += e.numel
        self.total = (off + _ALIGN - 1) // _ALIGN * _ALIGN
        self.by_key: Dict[str, Entry] = {e.key: e for e in self.entries}
        self.master: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.compute: Optional[torch.Tensor] = None
        self.compute_dtype = torch.float32
        self.params: Dict[str, nn.Parameter] = {}
        self._dirty = True
        # transposed bf16 working copies (Wᵀ) of selected 2-D weights, for NT-layout dgrad GEMMs
        self._t_keys: List[str] = []
        self._t_off: Dict[str, int] = {}
        self.compute_t: Optional[torch.Tensor] = None
        self._t_tiles: Optional[torch.Tensor] = None
        self._t_dirty = True
        self._fp8: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._fp8_state: Dict[str, object] = {}
        self._fp8_states_buf: Optional[torch.Tensor] = None
        self._fp8_dirty = True
        self._fp8_t_dirty = True   # e4m3 Wᵀ copies (fp8 dgrad GEMMs), transposed from the forward e4m3 bytes

    # ------------------------------------------------------------------ allocation
    def allocate(self, device, init_std: float, generator: Optional[torch.Generator] = None):
        self.master = torch.zeros(self.total, dtype=torch.float32, device="cpu")
        for e in self.entries:
            v = self.master[e.offset:e.offset + e.numel].view(e.shape)
            if e.init == "normal":
                v.normal_(0.0, init_std, generator=generator)
            elif e.init == "ones":
                v.fill_(1.0)
        self.master = self.master.to(device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        self._make_params()
        self.set_compute_dtype(self.compute_dtype)

    def _make_params(self):
        fresh = not self.params
        for e in self.entries:
            rows = e.shape[0]
            row_numel = e.numel // rows
            for hf_name, r0, r1 in e.views:
                shape = (r1 - r0,) + tuple(e.shape[1:])
                a = e.offset + r0 * row_numel
                b = e.offset + r1 * row_numel
                mv = self.master[a:b].view(shape)
                gv = self.grad[a:b].view(shape)
                if fresh:
                    p = nn.Parameter(mv, requires_grad=True)
                    self.params[hf_name] = p
                else:
                    p = self.params[hf_name]
                    p.data = mv
                p.grad = gv

    def set_compute_dtype(self, dtype: torch.dtype):
        self.compute_dtype = dtype
        if self.master is None:
            return
        if dtype == torch.float32:
            self.compute = self.master
        else:
            self.compute = torch.empty(self.total, dtype=dtype, device=self.master.device)
            self.compute.copy_(self.master)
        self._dirty = False
        self._t_dirty = True
        self._fp8_dirty = True
        self.compute_t = None
        self._t_tiles = None

    # ------------------------------------------------------------------ transposed copies
    def enable_transposed(self, keys: Sequence[str]):
        """Keep Wᵀ (bf16, [in, out] contiguous) for these 2-D entries on GPU, refreshed lazily after
        every change of the working copy (optimizer step, load, sync)."""
        self._t_keys = [k for k in keys if len(self.by_key[k].shape) == 2]
        off = 0
        for k in self._t_keys:
            self._t_off[k] = off
            off += (self.by_key[k].numel + _ALIGN - 1) // _ALIGN * _ALIGN
        self._t_total = off
        self._t_dirty = True

    def _transposable(self) -> bool:
        return (bool(self._t_keys) and self.compute is not None and self.compute.is_cuda
                and self.compute.dtype == torch.bfloat16)

    def refresh_transposed(self):
        from .._native import kernels
        if self.compute_t is None:
            self.compute_t = torch.empty(self._t_total, dtype=torch.bfloat16, device=self.compute.device)
        if self._t_tiles is None:
            rows = []
            for k in self._t_keys:
                e = self.by_key[k]
                R, Cc = e.shape
                assert R % 64 == 0 and Cc % 64 == 0, f"{k}: transposed copy needs 64-multiples, got {e.shape}"
                for r0 in range(0, R, 64):
                    for c0 in range(0, Cc, 64):
                        rows.append([e.offset, self._t_off[k], R, Cc, r0, c0])
            self._t_tiles = torch.tensor(rows, dtype=torch.int32).to(self.compute.device)
        kernels().transpose_tiles(self.compute, self.compute_t, self._t_tiles)
        self._t_dirty = False

    def view_fp8(self, key: str):
        """(W as float8_e4m3fn, dequant scale) of a registered weight for the fp8 forward GEMMs,
        re-quantised (current per-tensor scaling) after every change of the working copy."""
        if key not in self._t_off or not self._transposable():
            return None
        if self._fp8_dirty:
            self._requantize_fp8()
        return self._fp8[key]

    def _requantize_fp8(self):
        """Every registered weight -> e4m3 in ONE launch (gemm_fp8.hip quant_delayed_multi_kernel), each
        under its own delayed-scaling state (the amax of the previous update sets the scale); the first
        call seeds every state by current scaling.  Replaces one launch per weight (48 × ~13 µs)."""
        from .. import ops
        from .._native import kernels
        dev = self.compute.device
        if not self._fp8_state or self._fp8_states_buf.device != dev:
            n = len(self._t_keys)
            self._fp8_states_buf = torch.zeros(n, 4, dtype=torch.float32, device=dev)
            self._fp8_state = {kk: ops.Fp8DelayedState(dev, buf=self._fp8_states_buf[i])
                               for i, kk in enumerate(self._t_keys)}
            rows, yo, blk = [], 0, 0
            for kk in self._t_keys:
                e = self.by_key[kk]
                assert e.numel % 8 == 0 and e.offset % 8 == 0, f"{kk}: fp8 quantisation needs 8-aligned segments"
                rows.append([e.offset, yo, e.numel // 8, blk])
                blk += kernels().fp8_quant_multi_blocks(e.numel // 8)
                yo += (e.numel + 255) // 256 * 256
            self._fp8_seg = torch.tensor(rows, dtype=torch.int64).to(dev)
            self._fp8_blocks = blk
            self._fp8_y = torch.empty(yo, dtype=torch.uint8, device=dev)
            self._fp8_views = {kk: self._fp8_y[r[1]:r[1] + self.by_key[kk].numel].view(torch.float8_e4m3fn)
                               .view(self.by_key[kk].shape) for kk, r in zip(self._t_keys, rows)}
            self._fp8_step = 0
            for i, kk in enumerate(self._t_keys):   # seed: slot (0 + 2) % 3 = amax of the weight itself
                _, sc = kernels().fp8_quantize(self.view(kk))
                self._fp8_states_buf[i, 2] = sc.reshape(()) * 448.0
        phase = self._fp8_step % 3
        self._fp8_step += 1
        kernels().fp8_quant_delayed_multi(self.compute, self._fp8_y, self._fp8_seg, self._fp8_states_buf,
                                          self._fp8_blocks, phase)
        self._fp8 = {kk: (self._fp8_views[kk], self._fp8_state[kk].scale) for kk in self._t_keys}
        self._fp8_dirty = False
        self._fp8_t_dirty = True

    def view_fp8_t(self, key: str):
        """(Wᵀ as float8_e4m3fn [in, out], dequant scale) for the fp8 dgrad GEMMs: the bytes of the forward
        e4m3 copy transposed (one batched launch for every weight, after each re-quantisation), so forward
        and backward see the same quantised weight under the same scale."""
        from .._native import kernels
        if self.view_fp8(key) is None:
            return None
        if self._fp8_t_dirty:
            if getattr(self, "_fp8_ty", None) is None or self._fp8_ty.numel() != self._fp8_y.numel() \
                    or self._fp8_ty.device != self._fp8_y.device:
                self._fp8_ty = torch.empty_like(self._fp8_y)
                rows = []
                for kk, r in zip(self._t_keys, self._fp8_seg.tolist()):
                    R, Cc = self.by_key[kk].shape
                    for r0 in range(0, R, 64):
                        for c0 in range(0, Cc, 64):
                            rows.append([r[1], r[1], R, Cc, r0, c0])
                self._fp8_t_tiles = torch.tensor(rows, dtype=torch.int32).to(self._fp8_y.device)
                self._fp8_t_views = {kk: self._fp8_ty[r[1]:r[1] + self.by_key[kk].numel].view(torch.float8_e4m3fn)
                                     .view(self.by_key[kk].shape[1], self.by_key[kk].shape[0])
                                     for kk, r in zip(self._t_keys, self._fp8_seg.tolist())}
            kernels().transpose_tiles8(self._fp8_y, self._fp8_ty, self._fp8_t_tiles)
            self._fp8_t_dirty = False
        return self._fp8_t_views[key], self._fp8_state[key].scale

    def view_t(self, key: str) -> Optional[torch.Tensor]:
        """Wᵀ of a registered weight, or None when unavailable (CPU / fp32 / not registered)."""
        if key not in self._t_off or not self._transposable():
            return None
        if self._t_dirty:
            self.refresh_transposed()
        e = self.by_key[key]
        o = self._t_off[key]
        return self.compute_t[o:o + e.numel].view(e.shape[1], e.shape[0])

    def to(self, device):
        device = torch.device(device)
        if self.master is None or self.master.device == device:
            return self
        self.master = self.master.to(device)
        self.grad = self.grad.to(device)
        self._make_params()
        self.set_compute_dtype(self.compute_dtype if device.type == "cuda" else torch.float32)
        return self

    @property
    def device(self):
        return self.master.device

    # ------------------------------------------------------------------ views
    def view(self, key: str, which: str = "compute") -> torch.Tensor:
        e = self.by_key[key]
        buf = {"compute": self.compute, "master": self.master, "grad": self.grad}[which]
        return buf[e.offset:e.offset + e.numel].view(e.shape)

    def mark_master_dirty(self):
        self._dirty = True

    def sync_compute(self):
        """Refresh the bf16 working copy after host-side edits of master (load, init)."""
        if self._dirty and self.compute is not None and self.compute.data_ptr() != self.master.data_ptr():
            self.compute.copy_(self.master)
            self._t_dirty = True
            self._fp8_dirty = True
        self._dirty = False

    def mark_clean(self):
        """The optimizer rewrote master AND the working copy."""
        self._dirty = False
        self._t_dirty = True
        self._fp8_dirty = True

    # ------------------------------------------------------------------ layout queries
    def segments(self, names: Optional[Iterable[str]] = None) -> List[Tuple[int, int, str]]:
        """(start, numel, hf_name) for every HF parameter (optionally restricted to ``names``)."""
        wanted = None if names is None else set(names)
        out = []
        for e in self.entries:
            row_numel = e.numel // e.shape[0]
            for hf_name, r0, r1 in e.views:
                if wanted is not None and hf_name not in wanted:
                    continue
                out.append((e.offset + r0 * row_numel, (r1 - r0) * row_numel, hf_name))
        return out

    NORM_CHUNK = 1 << 18   # floats per grad-norm chunk (hq_kernels.h kNormChunk)

    def norm_chunks(self):
        """(chunk table int64 [C, 2] on the arena's device, {group: (c0, c1)}): every readiness group cut into pieces
        of <= NORM_CHUNK floats.  The grad norm is the fixed-order sum of one Σg² partial per chunk, so it is the same
        number whether the full pass computes every partial after the backward or the gradient reducer computes a
        bucket's partials on its comm stream right after that bucket's all-reduce."""
        cached = getattr(self, "_norm_chunks", None)
        if cached is not None and cached[0].device == self.grad.device:
            return cached
        rows, spans = [], {}
        for g, s, e in self.group_ranges():
            c0 = len(rows)
            for o in range(s, e, self.NORM_CHUNK):
                rows.append([o, min(self.NORM_CHUNK, e - o)])
            spans[g] = (c0, len(rows))
        self._norm_chunks = (torch.tensor(rows, dtype=torch.int64).to(self.grad.device), spans)
        return self._norm_chunks

    def group_ranges(self) -> List[Tuple[str, int, int]]:
        """Contiguous (group, start, end) ranges in arena order."""
        out: List[Tuple[str, int, int]] = []
        for e in self.entries:
            end = e.offset + e.numel
            if out and out[-1][0] == e.group:
                out[-1] = (e.group, out[-1][1], end)
            else:
                out.append((e.group, e.offset, end))
        # extend each range to the next range's start (covers alignment padding, keeps buckets contiguous)
        fixed = []
        for i, (g, s, _) in enumerate(out):
            e_ = out[i + 1][1] if i + 1 < len(out) else self.total
            fixed.append((g, s, e_))
        return fixed
