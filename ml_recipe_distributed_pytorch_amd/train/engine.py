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

Exact-objective merge (``merge_segments`` = G): the reference's micro-batches are collated one by one as it
does, then G of them run as one forward/backward whose loss scores each as its own segment — the same
gradient as G accumulated micro-steps (mean of per-micro-batch means), at merged-batch speed.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch

from .._native import kernels
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


def _tensors(data):
    if isinstance(data, (list, tuple)):
        for d in data:
            yield from _tensors(d)
    elif isinstance(data, dict):
        for d in data.values():
            yield from _tensors(d)
    elif torch.is_tensor(data):
        yield data


class DevicePrefetcher:
    """Host → device copies of upcoming batches on a copy stream, one batch ahead of the compute stream.

    A pinned-memory copy issued on the compute stream waited there behind the previous optimizer step: every step
    boundary left the GPU idle ~0.25 ms between the AdamW kernel and the next batch's first kernel while the runtime
    serviced the copies (``profiles/r6_s3/gaps_*.txt``, ``tools/trace_steps.py --gaps``).  Issued one batch early on
    their own stream, the copies run under the previous step's kernels and the compute stream only waits on an event
    that has long completed.  ``issue`` starts a copy, ``claim`` makes the current stream wait for it (and tells the
    caching allocator that stream uses the tensors).  On CPU both are plain ``to_device``."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def issue(self, data):
        if self.stream is None:
            return to_device(data, self.device), None
        # no wait on the compute stream: the copy must not queue behind the step it is meant to overlap (the
        # device buffers come from this stream's own pool, and the pinned source is the caller's to keep intact)
        with torch.cuda.stream(self.stream):
            dev = to_device(data, self.device)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dev, ev

    def claim(self, item):
        dev, ev = item
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            # a copy that has already landed (the usual case: it was issued a step early) needs no cross-queue
            # barrier packet in the compute stream (measured ~34 µs before the step's first kernel)
            if not ev.query():
                cur.wait_event(ev)
            for t in _tensors(dev):
                t.record_stream(cur)
        return dev


def prefetch_to_device(iterable, device):
    """Yield the items of ``iterable`` already on ``device``, each one's copy issued while the previous item is in
    use (``DevicePrefetcher``)."""
    pf = DevicePrefetcher(device)
    it = iter(iterable)
    try:
        nxt = pf.issue(next(it))
    except StopIteration:
        return
    for data in it:
        cur = pf.claim(nxt)
        nxt = pf.issue(data)
        yield cur
    yield pf.claim(nxt)


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
    """``graph=True`` (GPU, bf16 training, no grad side stream, fused QA heads): after two eager warm-up
    micro-steps, every kind of micro-step is captured once into a HIP graph and replayed for every later
    micro-batch of the same shape (inputs copied into the captured tensors, the dropout seed written to the
    model's device seed word).  A micro-step's kind is (fresh, sync):

    * fresh — the first micro-batch of an accumulation cycle overwrites the gradient arena (its graph also
      holds the Wᵀ refresh of the just-updated weights); later ones accumulate;
    * sync — the gradient reducer's bucket all-reduces run in it (the accumulation boundary, or every
      micro-batch with ``no_sync_accum=False``): RCCL collectives on the reducer's comm stream are captured
      as a fork/join of the capturing stream, so the 8-GPU DP step replays as one graph per micro-batch.

    So batch_split = 1 uses one graph, the reference's 128 × 2 accumulation three (first, middle, last).  The
    clip + fused optimizer step stays eager (its learning rate changes every step).  At small micro-batches
    the step is launch-bound (the reference's 2 × 512): one graph launch replaces ~300 kernel launches.

    Graphs are captured for at most ``max_graph_shapes`` distinct input shapes (the first ones seen); a
    micro-batch of any other shape (collate pads each NQ batch to its own length) runs eagerly beside them,
    so real data with many lengths cannot grow the graph set without bound.  Every capture allocates from
    ONE private mempool: the graphs replay one at a time on one stream, so a capture may reuse what an
    earlier one freed, and memory stays at about one micro-step's working set."""

    def __init__(self, model, loss_fn, optimizer, *, scheduler=None, reducer=None, max_grad_norm: float = 1.0,
                 batch_split: int = 1, no_sync_accum: bool = True, profile: bool = False, graph: bool = False,
                 max_graph_shapes: int = 2, merge_segments: int = 1):
        self.model = model
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.reducer = reducer
        self.max_grad_norm = max_grad_norm
        self.batch_split = max(1, int(batch_split))
        # exact-objective merge: every `merge_segments` consecutive micro-batches handed to micro_step() run as ONE
        # forward/backward whose loss keeps them as segments (data.collate.merge_micro_batches); `batch_split`
        # then counts those merged passes per optimizer step
        self.merge_segments = max(1, int(merge_segments))
        self._pending: List[tuple] = []
        self._pad_id = int(getattr(getattr(model, "config", None), "pad_token_id", 0) or 0)
        self.no_sync_accum = no_sync_accum
        self.profile = profile
        self.micro = 0
        self._timer = PhaseTimer(profile, model.store.device)
        self.graph = bool(graph)
        self._graphs: Dict[tuple, tuple] = {}   # (shape key, fresh, sync) -> (graph, static_in, static_lab, record)
        self._graph_shapes: List[tuple] = []    # shape keys with captured graphs, in capture order
        self.max_graph_shapes = max(1, int(max_graph_shapes))
        self._graph_pool = None                 # one private mempool shared by every capture
        self._graph_warm = 0
        self.graph_replays = 0
        self._steps = 0
        # optimizer steps between launches of the (asynchronous, sync-free) LayerNorm-from-y weight guard
        self.ln_check_every = 10
        self._ln_version = getattr(model, "ln_mode_version", 0)
        self.graph_eager_steps = 0              # micro-steps of an uncaptured shape run eagerly beside the graphs
        # --precision fp8: batch the ~97 per-site amax folds of a micro-step into a few launches at its end
        # (HQ_FP8_FOLD_DEFER=0: one fold launch per producing site, the immediate form)
        self.fp8_fold_defer = os.environ.get("HQ_FP8_FOLD_DEFER", "1") == "1"

    def _fp8_defer_folds(self) -> bool:
        return (self.fp8_fold_defer and getattr(self.model, "precision", "bf16") == "fp8"
                and self.model.store.device.type == "cuda")

    @property
    def device(self):
        return self.model.store.device

    # ------------------------------------------------------------------ HIP graph path
    def _graph_eligible(self) -> bool:
        from ..models.heads import fused_heads_possible
        m = self.model
        r = self.reducer
        return (self.graph and not self.profile and m.store.device.type == "cuda"
                and getattr(m, "precision", "bf16") == "bf16" and getattr(m, "grad_side_stream", None) is None
                and m.training
                # the reference-heads path draws its classifier dropout key on the host: a captured graph
                # would replay one mask forever (only the fused kernels read the device seed word)
                and fused_heads_possible(m)
                # the reducer's collectives are captured only on the native RCCL path (fence → ncclAllReduce on
                # its comm stream → join), the one the graph tests cover; the torch.distributed fallback
                # (work.wait(), gloo rescale) stays eager
                and (r is None or (r._native is not None and not r.timing and not r.verify)))

    @staticmethod
    def _shape_key(inputs, labels):
        """Tensor shapes/dtypes AND every non-tensor value (e.g. a merged batch's ``segment_lengths`` tuple):
        a replay refreshes only the captured tensors, so a host value the captured step read (the module-path
        loss slices each segment by its L_s) must select its own graph, never replay a stale one."""
        def part(k, v):
            if torch.is_tensor(v):
                return (k, tuple(v.shape), v.dtype)
            try:
                hash(v)
            except TypeError:
                v = repr(v)
            return (k, "value", v)
        return tuple(part(k, v) for d in (inputs, labels) for k, v in sorted(d.items()))

    def _kind(self):
        k = self.micro % self.batch_split
        fresh = k == 0
        boundary = k == self.batch_split - 1
        sync = self.reducer is not None and (boundary or not self.no_sync_accum)
        return fresh, sync, boundary

    def _set_fresh(self, fresh: bool):
        m = self.model
        if fresh:
            m.zero_grad()
        else:
            for g, _, _ in m.store.group_ranges():
                m._fresh[g] = False

    def _capture(self, inputs, labels, key, fresh: bool, sync: bool):
        m = self.model
        static_in = {k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()}
        static_lab = {k: v.clone() if torch.is_tensor(v) else v for k, v in labels.items()}
        m.use_device_seed(True)
        # the Wᵀ refresh of the updated weights belongs in the fresh (first micro-batch) graph only
        m.store._t_dirty = fresh
        self._set_fresh(fresh)
        if self.reducer is not None:
            self.reducer.prepare(sync=sync)
        side = torch.cuda.Stream(device=m.store.device)
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        rng = torch.get_rng_state()   # the capture's forward draws a (unused) host seed: keep the stream aligned
        with torch.cuda.graph(g, stream=side, pool=self._graph_pool):
            loss = self.loss_fn(m(**static_in), static_lab)
            self._backward(loss)
            if sync:
                self.reducer.finalize()   # the comm stream joins the capturing stream inside the graph
        torch.set_rng_state(rng)
        torch.cuda.current_stream().wait_stream(side)
        if self._graph_pool is None:
            self._graph_pool = g.pool()
        if key[0] not in self._graph_shapes:
            self._graph_shapes.append(key[0])
        self._graphs[key] = (g, static_in, static_lab, self.loss_fn.last)

    def _graph_capturable(self, inputs, labels) -> bool:
        shape = self._shape_key(inputs, labels)
        return shape in self._graph_shapes or len(self._graph_shapes) < self.max_graph_shapes

    def _graph_micro_step(self, inputs, labels) -> Optional[StepResult]:
        fresh, sync, boundary = self._kind()
        key = (self._shape_key(inputs, labels), fresh, sync)
        if key not in self._graphs:
            self._capture(inputs, labels, key, fresh, sync)
        g, static_in, static_lab, record = self._graphs[key]
        for src, dst in ((inputs, static_in), (labels, static_lab)):
            for k, v in src.items():
                if torch.is_tensor(v):
                    dst[k].copy_(v, non_blocking=True)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        self.model.seed_device.fill_(seed)
        if fresh:
            self._timer.reset()
        self._timer.mark()
        g.replay()
        self.graph_replays += 1
        # host-side state the replayed kernels changed: every gradient group now accumulates, Wᵀ is fresh
        self._set_fresh(False)
        if fresh:
            self.model.store._t_dirty = False
        self.loss_fn.last = record
        self._timer.mark("bwd")
        self.micro += 1
        if not boundary:
            return None
        return self._apply()

    def _check_ln_modes(self):
        """Fine-tuning moves γ / β: re-run the model's LayerNorm-from-y guard every ``ln_check_every`` steps —
        asynchronously (``poll_ln_modes``: device flags copied into pinned memory behind an event, applied at the
        next check, no host sync); a LayerNorm that changes mode invalidates the captured graphs."""
        from .. import ops
        poll = getattr(self.model, "poll_ln_modes", None)
        if poll is not None and ops.LN_FROM_Y:
            poll()
        self._sync_ln_version()

    def _sync_ln_version(self):
        """Release the graphs when the model's LayerNorm modes changed since they were captured (a guard check, or
        a ``load_state_dict`` — which re-runs the guard eagerly — between steps)."""
        v = getattr(self.model, "ln_mode_version", 0)
        if v != self._ln_version:
            self._ln_version = v
            if self._graphs:
                self.release_graph()

    def release_graph(self):
        if self._graphs:
            self.model.use_device_seed(False)
        self._graphs, self._graph_warm = {}, 0
        self._graph_shapes, self._graph_pool = [], None

    def micro_step(self, inputs, labels) -> Optional[StepResult]:
        """Forward+backward of one micro-batch; runs the optimizer on the accumulation boundary.  With
        ``merge_segments`` = G > 1 the micro-batches are buffered and every G of them run as one merged pass."""
        if self.merge_segments > 1:
            self._pending.append((inputs, labels))
            if len(self._pending) < self.merge_segments:
                return None
            from ..data.collate import merge_micro_batches
            inputs, labels = merge_micro_batches(self._pending, self._pad_id)
            self._pending = []
        return self._pass(inputs, labels)

    def _pass(self, inputs, labels) -> Optional[StepResult]:
        self._sync_ln_version()
        if self._graph_eligible():
            if (self._graph_warm >= 2 or self._graphs) and self._graph_capturable(inputs, labels):
                return self._graph_micro_step(inputs, labels)
            if not self._graphs:
                self._graph_warm += 1   # eager warm-up: kernel attributes, Wᵀ copies, allocator pools
        elif self._graphs:
            self.release_graph()
        if self._graphs:   # eager step beside live graphs (an uncaptured shape): host seeds again
            self.graph_eager_steps += 1
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
        defer = self._fp8_defer_folds()
        if defer:   # the fp8 sites' amax folds run batched at the end of the micro-step (gemm_fp8.hip, FoldDefer)
            kernels().fp8_fold_defer(True)
        try:
            preds = self.model(**inputs)
            loss = self.loss_fn(preds, labels)
            timer.mark("fwd")
            self._backward(loss)
        finally:
            if defer:
                kernels().fp8_fold_defer(False)   # launches the pending folds
        if self.reducer is not None and not boundary and not self.no_sync_accum:
            self.reducer.finalize()
        timer.mark("bwd")
        self.micro += 1
        if not boundary:
            return None
        return self._apply()

    def _backward(self, loss):
        """(loss / batch_split).backward() without the two scalar kernels and the ones-fill autograd would launch:
        the seed gradient d(loss/S)/d(loss) = 1/S is a cached device scalar (computed once as fp32 1/S — the same
        value DivBackward produces)."""
        seed = getattr(self, "_grad_seed", None)
        if (seed is None or seed.device != loss.device or seed.dtype != loss.dtype
                or getattr(self, "_grad_seed_split", None) != self.batch_split):
            seed = (torch.ones((), dtype=torch.float32) / self.batch_split).to(loss.dtype).to(loss.device)
            self._grad_seed, self._grad_seed_split = seed, self.batch_split
        torch.autograd.backward(loss, grad_tensors=seed)

    def _apply(self) -> StepResult:
        timer = self._timer
        side = getattr(self.model, "grad_side_stream", None)
        if side is not None:  # weight grads from the side stream must be complete
            torch.cuda.current_stream().wait_stream(side)
        if self.reducer is not None:
            self.reducer.finalize()
            if self.reducer.snapshot_grads:   # replica check: fingerprint the reduced gradients (untimed steps only)
                self.reducer.take_grad_snapshot()
        timer.mark("comm_wait")
        parts = self.reducer.norm_partials() if self.reducer is not None else None
        norm, coef = grad_norm_and_clip(self.model.store, self.max_grad_norm, partials=parts)
        lr = self.optimizer.param_groups[0]["lr"]
        self.optimizer.step(clip_coef=coef)
        self.optimizer.zero_grad()
        if self.scheduler is not None:
            self.scheduler.step()
        timer.mark("optim")
        self._steps += 1
        if self._steps % self.ln_check_every == 0 and self.device.type == "cuda":
            self._check_ln_modes()
        return StepResult(losses=self.loss_fn.last, grad_norm=norm, lr=lr, timings=timer.resolve())

    def step(self, micro_batches) -> StepResult:
        res = None
        for inputs, labels in micro_batches:
            res = self.micro_step(inputs, labels)
        assert res is not None, "number of micro-batches must equal batch_split × merge_segments"
        return res
