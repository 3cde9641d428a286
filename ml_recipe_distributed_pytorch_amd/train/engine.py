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
    """``graph=True`` (GPU, bf16, one micro-batch per step, no gradient reducer): after two eager warm-up
    steps the forward + loss + backward of a micro-batch is captured once into a HIP graph and replayed for
    every later batch of the same shape (inputs copied into the captured tensors, the dropout seed written
    to the model's device seed word); the clip + fused optimizer step stays eager (its learning rate
    changes every step).  At small micro-batches the step is launch-bound (the reference's 2 × 512):
    one graph launch replaces ~300 kernel launches.  Other shapes fall back to the eager path."""

    def __init__(self, model, loss_fn, optimizer, *, scheduler=None, reducer=None, max_grad_norm: float = 1.0,
                 batch_split: int = 1, no_sync_accum: bool = True, profile: bool = False, graph: bool = False):
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
        self.graph = bool(graph)
        self._graph = None
        self._graph_warm = 0
        self._static = None
        self.graph_replays = 0

    @property
    def device(self):
        return self.model.store.device

    # ------------------------------------------------------------------ HIP graph path
    def _graph_eligible(self) -> bool:
        m = self.model
        return (self.graph and self.batch_split == 1 and self.reducer is None and not self.profile
                and m.store.device.type == "cuda" and getattr(m, "precision", "bf16") == "bf16"
                and getattr(m, "grad_side_stream", None) is None and m.training)

    @staticmethod
    def _shape_key(inputs, labels):
        return tuple((k, tuple(v.shape), v.dtype) for d in (inputs, labels) for k, v in sorted(d.items())
                     if torch.is_tensor(v))

    def _capture(self, inputs, labels):
        m = self.model
        static_in = {k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()}
        static_lab = {k: v.clone() if torch.is_tensor(v) else v for k, v in labels.items()}
        m.use_device_seed(True)
        m.store._t_dirty = True   # the Wᵀ refresh belongs in the graph: the weights change every step
        m.zero_grad()             # "fresh" groups: the captured backward overwrites the arena gradients
        side = torch.cuda.Stream(device=m.store.device)
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        rng = torch.get_rng_state()   # the capture's forward draws a (unused) host seed: keep the stream aligned
        with torch.cuda.graph(g, stream=side):
            loss = self.loss_fn(m(**static_in), static_lab)
            loss.backward()
        torch.set_rng_state(rng)
        torch.cuda.current_stream().wait_stream(side)
        self._graph, self._static = g, (static_in, static_lab, self._shape_key(inputs, labels), self.loss_fn.last)

    def _graph_micro_step(self, inputs, labels) -> Optional[StepResult]:
        if self._graph is None:
            if self._graph_warm < 2:          # eager warm-up: kernel attributes, Wᵀ copies, allocator pools
                self._graph_warm += 1
                return None
            self._capture(inputs, labels)
        elif self._shape_key(inputs, labels) != self._static[2]:
            return None
        static_in, static_lab, _, record = self._static
        for src, dst in ((inputs, static_in), (labels, static_lab)):
            for k, v in src.items():
                if torch.is_tensor(v):
                    dst[k].copy_(v, non_blocking=True)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        self.model.seed_device.fill_(seed)
        self._timer.reset()
        self._timer.mark()
        self._graph.replay()
        self.graph_replays += 1
        self.loss_fn.last = record
        self._timer.mark("bwd")
        self.micro += 1
        return self._apply()

    def release_graph(self):
        if self._graph is not None:
            self.model.use_device_seed(False)
        self._graph, self._static, self._graph_warm = None, None, 0

    def micro_step(self, inputs, labels) -> Optional[StepResult]:
        """Forward+backward of one micro-batch; runs the optimizer on the accumulation boundary."""
        if self._graph_eligible():
            res = self._graph_micro_step(inputs, labels)
            if res is not None:
                return res
        elif self._graph is not None:
            self.release_graph()
        if self._graph is not None:   # eager step beside a live graph: host seeds again
            self.model.use_device_seed(False)
            try:
                return self._eager_micro_step(inputs, labels)
            finally:
                self.model.use_device_seed(True)
        return self._eager_micro_step(inputs, labels)

    def _eager_micro_step(self, inputs, labels) -> Optional[StepResult]:
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
