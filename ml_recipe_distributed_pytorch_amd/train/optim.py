"""Fused arena optimizers: HF-semantics AdamW and AdaMod over the flat fp32 master arena.

* ``FusedAdamW`` = ``transformers.AdamW`` as used by the reference (``modules/init.py:137``:
  ``AdamW(groups, lr, correct_bias=False)``, eps 1e-6, decoupled decay applied after the update;
  transformers 5.x dropped the class — SURVEY D18).
* ``FusedAdaMod`` = reference ``modules/model/trainer/optim.py:8-100`` (decay before the update,
  beta3 EMA bound on the per-element step size), rewritten without the removed ``add_(scalar, t)``
  overloads (D17).

Both are ``torch.optim.Optimizer`` subclasses (so ``LambdaLR`` and ``state_dict()`` work and the
checkpoint layout matches the reference: per-param ``step/exp_avg/exp_avg_sq``), but their state
tensors are *views* into flat arenas and ``step()`` is ONE kernel on GPU (``_hq_kernels.adamw``)
that also reads the on-device clip coefficient and refreshes the bf16 working copy.  On CPU the
same arithmetic runs in ``ops.reference``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .._native import kernels
from ..models.params import ParamStore
from ..ops import reference as ref

CHUNK = 8192


class _ArenaOptimizer(torch.optim.Optimizer):
    state_names: Tuple[str, ...] = ()

    def __init__(self, params, defaults, store: ParamStore, zero_grad_fn=None):
        super().__init__(params, defaults)
        self.store = store
        self._zero_grad_fn = zero_grad_fn
        self._arenas: Dict[str, torch.Tensor] = {}
        self._chunks: Optional[torch.Tensor] = None
        self._segments: List[Tuple[int, int, int]] = []   # (start, numel, group)
        self._index_params()

    # ----------------------------------------------------------------------------- layout
    def _index_params(self):
        addr = {}
        base = self.store.master.data_ptr()
        for start, numel, name in self.store.segments():
            addr[base + 4 * start] = (start, numel)
        segs = []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                key = p.data_ptr()
                if key not in addr:
                    raise ValueError("FusedOptimizer only manages parameters that live in the model's arena")
                s, n = addr[key]
                segs.append((s, n, gi))
        segs.sort()
        self._segments = segs
        self._chunks = None

    def _arena(self, name: str) -> torch.Tensor:
        t = self._arenas.get(name)
        dev = self.store.master.device
        if t is None or t.device != dev:
            old = t
            t = torch.zeros_like(self.store.master)
            if old is not None:
                t.copy_(old)
            self._arenas[name] = t
            self._bind_state()
        return t

    def _bind_state(self):
        """Point every param's state entries at its slice of the arenas."""
        base = self.store.master.data_ptr()
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state[p]
                off = (p.data_ptr() - base) // 4
                n = p.numel()
                for name, arena in self._arenas.items():
                    st[name] = arena[off:off + n].view_as(p)
                st.setdefault("step", 0)

    def _chunk_table(self) -> torch.Tensor:
        dev = self.store.master.device
        if self._chunks is None or self._chunks.device != dev:
            rows = []
            for s, n, g in self._segments:
                for off in range(0, n, CHUNK):
                    rows.append([s + off, min(CHUNK, n - off) | (g << 32)])
            self._chunks = torch.tensor(rows, dtype=torch.int64).to(dev)
        return self._chunks

    def _sync_device(self):
        if self.store.master.device.type == "cuda":
            for name in self.state_names:
                self._arena(name)
            self._chunk_table()

    # ----------------------------------------------------------------------------- API
    def zero_grad(self, set_to_none: bool = False):
        if self._zero_grad_fn is not None:
            self._zero_grad_fn()
        else:
            self.store.grad.zero_()

    def _step_count(self) -> int:
        first = self.param_groups[0]["params"][0]
        return int(self.state[first].get("step", 0))

    def _bump_steps(self):
        for group in self.param_groups:
            for p in group["params"]:
                self.state[p]["step"] = int(self.state[p].get("step", 0)) + 1

    def load_state_dict(self, state_dict):
        saved = {}
        for idx, st in state_dict.get("state", {}).items():
            saved[idx] = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
        super().load_state_dict(state_dict)
        for name in self.state_names:
            self._arena(name)
        self._bind_state()
        idx = 0
        for group in self.param_groups:
            for p in group["params"]:
                st = saved.get(idx) or saved.get(str(idx))
                if st is not None:
                    for name in self.state_names:
                        if name in st:
                            self.state[p][name].copy_(st[name].to(p.device).view_as(p))
                    step = st.get("step", 0)
                    self.state[p]["step"] = int(step.item() if torch.is_tensor(step) else step)
                idx += 1


class FusedAdamW(_ArenaOptimizer):
    state_names = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, store: ParamStore, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-6,
                 weight_decay: float = 0.0, correct_bias: bool = True, zero_grad_fn=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, correct_bias=correct_bias)
        super().__init__(params, defaults, store, zero_grad_fn)
        for name in self.state_names:
            self._arena(name)

    @torch.no_grad()
    def step(self, closure=None, clip_coef: Optional[torch.Tensor] = None):
        loss = closure() if closure is not None else None
        self._sync_device()
        self._bump_steps()
        step = self._step_count()
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        mult = math.sqrt(1.0 - b2 ** step) / (1.0 - b1 ** step) if g0["correct_bias"] else 1.0
        st = self.store
        if st.master.is_cuda:
            compute = st.compute if st.compute.data_ptr() != st.master.data_ptr() else None
            kernels().adamw(st.master, compute, st.grad, self._arenas["exp_avg"], self._arenas["exp_avg_sq"],
                            self._chunk_table(), [g["lr"] for g in self.param_groups],
                            [g["weight_decay"] for g in self.param_groups], b1, b2, g0["eps"], mult, clip_coef)
        else:
            for gi, g in enumerate(self.param_groups):
                segs = [(s, n, g["weight_decay"]) for s, n, gg in self._segments if gg == gi]
                ref.adamw_step(st.master, None, st.grad, self._arenas["exp_avg"], self._arenas["exp_avg_sq"], segs,
                               lr=g["lr"], beta1=b1, beta2=b2, eps=g["eps"], clip_coef=clip_coef,
                               correct_bias=g["correct_bias"], step=step)
        st.mark_clean()
        return loss


class FusedAdaMod(_ArenaOptimizer):
    state_names = ("exp_avg", "exp_avg_sq", "exp_avg_lr")

    def __init__(self, params, store: ParamStore, lr: float = 1e-3, betas=(0.9, 0.999), beta3: float = 0.999,
                 eps: float = 1e-8, weight_decay: float = 0.0, zero_grad_fn=None):
        defaults = dict(lr=lr, betas=betas, beta3=beta3, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults, store, zero_grad_fn)
        for name in self.state_names:
            self._arena(name)

    @torch.no_grad()
    def step(self, closure=None, clip_coef: Optional[torch.Tensor] = None):
        loss = closure() if closure is not None else None
        self._sync_device()
        self._bump_steps()
        step = self._step_count()
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        bias = math.sqrt(1.0 - b2 ** step) / (1.0 - b1 ** step)
        st = self.store
        if st.master.is_cuda:
            compute = st.compute if st.compute.data_ptr() != st.master.data_ptr() else None
            kernels().adamod(st.master, compute, st.grad, self._arenas["exp_avg"], self._arenas["exp_avg_sq"],
                             self._arenas["exp_avg_lr"], self._chunk_table(), [g["lr"] for g in self.param_groups],
                             [g["weight_decay"] for g in self.param_groups], b1, b2, g0["beta3"], g0["eps"], bias,
                             clip_coef)
        else:
            for gi, g in enumerate(self.param_groups):
                segs = [(s, n, g["weight_decay"]) for s, n, gg in self._segments if gg == gi]
                ref.adamod_step(st.master, None, st.grad, self._arenas["exp_avg"], self._arenas["exp_avg_sq"],
                                self._arenas["exp_avg_lr"], segs, lr=g["lr"], beta1=b1, beta2=b2, beta3=g["beta3"],
                                eps=g["eps"], clip_coef=clip_coef, step=step)
        st.mark_clean()
        return loss


def grad_norm_and_clip(store: ParamStore, max_norm: float, partials: Optional[torch.Tensor] = None):
    """Global L2 norm of the grad arena + clip coefficient, both as device scalars (no host sync).
    Matches ``torch.nn.utils.clip_grad_norm_`` (coef = max_norm / (norm + 1e-6), clamped to 1).
    GPU: one Σg² partial per chunk of ``store.norm_chunks()`` then a fixed-order fold; ``partials`` = a complete
    vector already written (the gradient reducer's comm stream computes each bucket's partials right after its
    all-reduce, so the step tail is only the fold) — bitwise the same result as the full pass."""
    g = store.grad
    if g.is_cuda:
        if partials is None:
            chunks, _ = store.norm_chunks()
            partials = torch.empty(chunks.shape[0], dtype=torch.float32, device=g.device)
            kernels().sq_norm_chunks(g, chunks, 0, chunks.shape[0], partials)
        norm, coef = kernels().clip_from_partials(partials, float(max_norm))
        return norm, (coef if max_norm > 0 else None)
    norm = g.float().norm()
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else None
    return norm, coef


def linear_schedule_with_warmup(num_warmup_steps: int, num_training_steps: int):
    """LR multiplier of transformers' ``get_linear_schedule_with_warmup`` (reference trainer.py:116-126)."""
    def fn(step: int) -> float:
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        return max(0.0, float(num_training_steps - step) / float(max(1, num_training_steps - num_warmup_steps)))
    return fn


def get_linear_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int, last_epoch: int = -1):
    """The multiplier is a plain closure on purpose: ``LambdaLR.state_dict`` serialises the ``__dict__`` of
    callable *objects* and ``load_state_dict`` writes it back, so a resumed run with more epochs would
    inherit the old (warmup, total) and train at LR 0.  Functions are not serialised, so a resume keeps
    the current run's schedule (as with transformers' lambda in the reference)."""
    return torch.optim.lr_scheduler.LambdaLR(optimizer, linear_schedule_with_warmup(num_warmup_steps, num_training_steps),
                                             last_epoch)
