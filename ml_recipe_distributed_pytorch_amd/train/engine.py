"""One optimizer step of QA fine-tuning: the hot loop shared by ``Trainer`` and ``bench.py``.

Per optimizer step (reference ``trainer.py:266-300`` semantics, re-engineered):
  for each of ``batch_split`` micro-batches:
      reducer.prepare(sync = last micro-batch)        # no_sync accumulation (fix of D1)
      preds = model(**inputs); loss = Σ w_k·loss_k    # fused encoder, fp32 heads
      (loss / batch_split).backward()                 # layer backward → arena grads → bucket all-reduce
  reducer.finalize()                                  # compute stream waits for the last bucket
  norm, coef = grad_norm_and_clip(arena)              # device scalars, no host sync
  optimizer.step(clip_coef=coef)                      # one fused AdamW kernel (+ bf16 copy-out)
  optimizer.zero_grad(); scheduler.step()
Loss values stay on device (``LossRecord``); callers sync them at their logging cadence.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch

from ..models.losses import LossRecord
from .optim import grad_norm_and_clip


def to_device(data, device, non_blocking=True):
    if isinstance(data, (list, tuple)):
        return [to_device(d, device, non_blocking) for d in data]
    if isinstance(data, dict):
        return {k: to_device(v, device, non_blocking) for k, v in data.items()}
    if torch.is_tensor(data):
        return data.to(device, non_blocking=non_blocking)
    return data


class PhaseTimer:
    """Per-phase step timer.  On GPU it records HIP events on the compute stream (no per-phase
    synchronisation; ``resolve`` waits for the last event once per step, profiling runs only);
    on CPU it reads the wall clock.  Phases repeated across micro-batches are summed."""

    def __init__(self, enabled: bool, device):
        self.enabled = enabled
        self.cuda = torch.device(device).type == "cuda"
        self.marks: List = []

    def reset(self):
        self.marks = []

    def mark(self, name: str = "start"):
        if not self.enabled:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.marks.append((name, ev))
        else:
            self.marks.append((name, time.perf_counter()))

    def resolve(self) -> Dict[str, float]:
        if not self.enabled or len(self.marks) < 2:
            return {}
        if self.cuda:
            self.marks[-1][1].synchronize()
        out: Dict[str, float] = {}
        for (_, a), (name, b) in zip(self.marks, self.marks[1:]):
            if name == "start":
                continue
            ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
            out[name + "_ms"] = out.get(name + "_ms", 0.0) + ms
        return out


@dataclass
class StepResult:
    losses: LossRecord
    grad_norm: Optional[torch.Tensor]
    lr: float
    timings: Dict[str, float] = field(default_factory=dict)


class TrainEngine:
    def __init__(self, model, loss_fn, optimizer, *, scheduler=None, reducer=None, max_grad_norm: float = 1.0,
                 batch_split: int = 1, no_sync_accum: bool = True, profile: bool = False):
        self.model = model
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.reducer = reducer
        self.max_grad_norm = max_grad_norm
        self.batch_split = max(1, int(batch_split))
        self.no_sync_accum = no_sync_accum
        self.profile = profile
        self.micro = 0
        self._timer = PhaseTimer(profile, model.store.device)

    @property
    def device(self):
        return self.model.store.device

    def micro_step(self, inputs, labels) -> Optional[StepResult]:
        """Forward+backward of one micro-batch; runs the optimizer on the accumulation boundary."""
        timer = self._timer
        if self.micro % self.batch_split == 0:
            timer.reset()
        timer.mark()
        boundary = (self.micro + 1) % self.batch_split == 0
        if self.reducer is not None:
            self.reducer.prepare(sync=boundary or not self.no_sync_accum)
        preds = self.model(**inputs)
        loss = self.loss_fn(preds, labels)
        timer.mark("fwd")
        (loss / self.batch_split).backward()
        if self.reducer is not None and not boundary and not self.no_sync_accum:
            self.reducer.finalize()
        timer.mark("bwd")
        self.micro += 1
        if not boundary:
            return None
        return self._apply()

    def _apply(self) -> StepResult:
        timer = self._timer
        side = getattr(self.model, "grad_side_stream", None)
        if side is not None:  # weight grads from the side stream must be complete
            torch.cuda.current_stream().wait_stream(side)
        if self.reducer is not None:
            self.reducer.finalize()
        timer.mark("comm_wait")
        norm, coef = grad_norm_and_clip(self.model.store, self.max_grad_norm)
        lr = self.optimizer.param_groups[0]["lr"]
        self.optimizer.step(clip_coef=coef)
        self.optimizer.zero_grad()
        if self.scheduler is not None:
            self.scheduler.step()
        timer.mark("optim")
        return StepResult(losses=self.loss_fn.last, grad_norm=norm, lr=lr, timings=timer.resolve())

    def step(self, micro_batches) -> StepResult:
        res = None
        for inputs, labels in micro_batches:
            res = self.micro_step(inputs, labels)
        assert res is not None, "number of micro-batches must equal batch_split"
        return res
