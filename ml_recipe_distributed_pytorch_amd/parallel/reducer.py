"""Data-parallel gradient reducer over the flat grad arena (replaces torch DDP).

Buckets are contiguous arena ranges built from the model's readiness groups (QA head+pooler,
layer N-1 … layer 0, embeddings — the order backward produces them), merged until each reaches
``bucket_cap_mb``.  The fused layer backward calls ``_on_group_ready``; when every group of a
bucket has reported, the bucket's all-reduce is issued immediately, so communication overlaps
the remaining backward.  ``finalize()`` makes the compute stream wait for the last bucket.

* GPU + nccl: the native C++ ``Reducer`` owns an RCCL communicator and a normal-priority comm
  stream; ncclAvg in place on the arena slice (fp32) or through a bf16 scratch (``allreduce_dtype``:
  ``fp32`` | ``bf16`` for every bucket | ``emb_bf16`` — only the embeddings bucket in bf16: the 89 MiB word-
  embedding gradient is produced by the LAST backward kernel, so its all-reduce is the one exposed tail of
  the step; halving its bytes halves that tail while every other bucket stays exact fp32).
* CPU / gloo (and GPU when ``native=False``): ``torch.distributed.all_reduce(async_op=True)``.
* ``prepare(sync=False)`` = DDP ``no_sync``: no communication during accumulation micro-batches
  (fixes reference D1, which all-reduced every micro-batch).
* ``kind`` says which path runs ("native-rccl" | "torch-nccl" | "torch-gloo" | "none") and bench.py
  reports it.  A failing native RCCL init is FATAL on an nccl process group (an 8-GPU number must never
  silently measure the fallback); ``HQ_REDUCER_FALLBACK=1`` opts into the torch.distributed path.
* ``force=True`` keeps the reducer active at world size 1 (a 1-rank RCCL communicator): every bucket of
  a real backward goes through fence → ncclAllReduce → wait, which is how one GPU rehearses the 8-GPU
  path (bench.py ``--force_reducer``; tests/test_kernels_gpu.py checks bitwise-equal weights).
* ``verify=True`` (or ``HQ_REDUCER_VERIFY=1``): the comm stream also records a deterministic checksum of
  every bucket at the exact point its all-reduce reads it; ``check_order()`` compares them with the final
  gradients — a bucket read before its (side-stream) weight-gradient GEMMs finished shows up as a mismatch.
* Grad-norm partials (native path): right after a bucket's all-reduce (and bf16 cast-back) the comm stream writes
  the Σg² partials of that bucket's chunks (``ParamStore.norm_chunks``), so when the last bucket lands the clip
  coefficient needs one tiny fold instead of a pass over the whole 418 MiB arena on the step's critical path
  (``norm_partials()``; bitwise the same coefficient as the full pass, ``train/optim.grad_norm_and_clip``).
* ``timing=True``: HIP events on the compute and comm streams give the comm span and the EXPOSED wait
  (comm still running after the backward's last kernel) per synchronised step (``pop_timings()``).

Sizing for xGMI: MI355X peers are point-to-point links (7 × ~153 GB/s per GPU); RCCL splits a
bucket over its channels/rings, so 32 MiB buckets give each channel multi-MiB chunks while the first
bucket (heads + last layer, ~30 MB) still starts early in the backward.
"""
from __future__ import annotations

import itertools
import logging
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .._native import kernels

logger = logging.getLogger(__name__)
_uid_counter = itertools.count()


def _part_bounds(n: int, parts: int):
    return [(n * p // parts, n * (p + 1) // parts) for p in range(parts)]


def fingerprint(x: torch.Tensor, parts: int = 256) -> torch.Tensor:
    """Exact fingerprint of an fp32 tensor: ``parts`` int64 words, word p = Σ bits(x_i)·(2i+1) mod 2^64 over the
    p-th contiguous slice (i = global index).  Integer wrap-around sums do not depend on summation order, so the
    GPU kernel (``optim.hip`` ``fingerprint_kernel``) and this host path give the same bits; any changed bit,
    sign or swapped pair of words changes the word of its slice."""
    x = x.detach().contiguous().view(-1)
    assert x.dtype == torch.float32
    if x.is_cuda:
        return kernels().fingerprint(x, parts)
    import numpy as np
    a = x.view(torch.int32).numpy().view(np.uint32)
    out = np.zeros(parts, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for p, (lo, hi) in enumerate(_part_bounds(a.size, parts)):
            i = np.arange(lo, hi, dtype=np.uint64)
            out[p] = np.sum(a[lo:hi].astype(np.uint64) * (np.uint64(2) * i + np.uint64(1)), dtype=np.uint64)
    return torch.from_numpy(out.view(np.int64))


def sq_partials(x: torch.Tensor, parts: int = 256) -> torch.Tensor:
    """Σx² per contiguous slice (the same slices as ``fingerprint``), float64 on the host: the magnitude of a
    replica mismatch (the fingerprint says only whether the bits differ)."""
    x = x.detach().contiguous().view(-1).double().cpu()
    return torch.stack([x[lo:hi].square().sum() for lo, hi in _part_bounds(x.numel(), parts)])


class Bucket:
    __slots__ = ("index", "start", "end", "groups", "pending", "launched", "work", "dtype")

    def __init__(self, index, start, end, groups, dtype="fp32"):
        self.index, self.start, self.end, self.groups = index, start, end, list(groups)
        self.dtype = dtype
        self.pending = len(self.groups)
        self.launched = False
        self.work = None

    @property
    def numel(self):
        return self.end - self.start


class GradReducer:
    def __init__(self, model, *, bucket_cap_mb: float = 32.0, allreduce_dtype: str = "fp32",
                 native: Optional[bool] = None, broadcast_params: bool = True, group=None, force: bool = False,
                 verify: Optional[bool] = None, timing: bool = False):
        self.model = model
        self.store = model.store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.bucket_cap = int(bucket_cap_mb * 1024 * 1024)
        self.allreduce_dtype = allreduce_dtype
        self.force = bool(force)
        self.active = False
        self.buckets: List[Bucket] = []
        self._bucket_chunks: Dict[int, Tuple[int, int]] = {}
        self.group_to_bucket: Dict[str, Bucket] = {}
        self._native = None
        self._scratch = None
        self.uid_via_store = False
        self.broadcast_done = False
        self.stats = {"buckets_launched": 0, "bytes": 0}
        self._seq_hash = 0       # running hash of the (bucket, numel) launch sequence (SURVEY §5.2 checker)
        # replica check: with ``snapshot_grads`` set, the engine fingerprints the REDUCED gradient arena of the next
        # optimizer step (after finalize, before zero_grad) — bench.py sets it for one untimed step after the clock
        self.snapshot_grads = False
        self._grad_fp: Optional[torch.Tensor] = None
        self._grad_sq: Optional[torch.Tensor] = None
        on_gpu = self.store.device.type == "cuda"
        backend = dist.get_backend(group) if dist.is_initialized() else None
        if native is None:
            native = on_gpu and (backend == "nccl" or (self.force and self.world == 1))
        self.kind = "none"
        if (self.world > 1 or self.force) and native:
            try:
                self._native = self._make_native()
                self.kind = "native-rccl"
            except Exception as e:
                if os.environ.get("HQ_REDUCER_FALLBACK", "0") != "1" or self.world == 1:
                    raise RuntimeError(f"native RCCL reducer failed to initialise: {e} "
                                       "(HQ_REDUCER_FALLBACK=1 allows the torch.distributed path)") from e
                logger.warning(f"native RCCL reducer unavailable ({e}); HQ_REDUCER_FALLBACK=1 → torch.distributed")
                self._native = None
        if self._native is None and self.world > 1:
            self.kind = f"torch-{backend}"
        if verify is None:
            verify = os.environ.get("HQ_REDUCER_VERIFY", "0") == "1"
        self.verify = bool(verify) and self._native is not None
        self._probes: Dict[int, torch.Tensor] = {}
        self.timing = bool(timing) and self._native is not None
        self._tev: List[tuple] = []
        self._first_ev = None
        self._build_buckets()
        self._norm_parts = None
        self._norm_ready = False
        if self._native is not None:
            chunks, spans = self.store.norm_chunks()
            self._norm_chunks = chunks
            self._norm_parts = torch.zeros(chunks.shape[0], dtype=torch.float32, device=self.store.device)
            for b in self.buckets:   # a bucket's groups are consecutive arena ranges -> one contiguous chunk run
                cs = [spans[g] for g in b.groups]
                b_c0, b_c1 = min(c[0] for c in cs), max(c[1] for c in cs)
                assert b_c1 - b_c0 == sum(c[1] - c[0] for c in cs), "bucket groups must be contiguous"
                self._bucket_chunks[b.index] = (b_c0, b_c1)
            # chunks of groups that no bucket carries (frozen parameters): computed on the compute stream at finalize
            self._uncovered, at = [], 0
            for c0, c1 in sorted(self._bucket_chunks.values()):
                if c0 > at:
                    self._uncovered.append((at, c0))
                at = max(at, c1)
            if at < chunks.shape[0]:
                self._uncovered.append((at, int(chunks.shape[0])))
        model.set_grad_listener(self._on_group_ready)
        self.gemm_sched = self._pick_gemm_sched(on_gpu)
        # DDP-constructor broadcast whenever a process group exists (any world size: a 1-rank
        # torchrun rehearsal runs the same native ncclBroadcast an 8-GPU job does) or the reducer is forced
        self.broadcast_done = False
        if broadcast_params and (self.world > 1 or (self.force and (dist.is_initialized() or self._native is not None))):
            self.broadcast_parameters()

    # ------------------------------------------------------------------ setup
    def _pick_gemm_sched(self, on_gpu: bool) -> str:
        """Persistent-GEMM tile schedule while gradients are all-reduced under the backward: the collective's
        blocks hold CUs, and with the static schedule the GEMM workgroups that wait for those CUs run their
        whole share late (+160-180 µs per GEMM per 200 µs held, tools/gemm_contention_bench.py); the dynamic
        per-XCD ticket schedule costs ~0.9 % of the uncontended step, so it is switched on only here, when a
        collective actually overlaps the backward — or when ``force`` rehearses that path on one GPU.
        HQ_GEMM_SCHED (0/1) overrides."""
        if not on_gpu:
            return "n/a"
        env = os.environ.get("HQ_GEMM_SCHED")
        dynamic = (env == "1") if env in ("0", "1") else (self.world > 1 or self.force)
        kernels().gemm_set_sched(1 if dynamic else 0)
        self._set_sched = dynamic
        return "dynamic" if dynamic else "static"

    def _make_native(self):
        """RCCL communicator over this group's ranks.  Whenever a process group exists (also at world 1 under
        torchrun) rank 0's unique id travels through the rendezvous TCPStore, so a 1-rank
        rehearsal executes the same exchange as an 8-rank job; only a forced reducer without any process
        group creates its id locally.  ``uid_via_store`` records which one ran."""
        self.uid_via_store = False
        if not dist.is_initialized():   # forced single-rank communicator, no process group: nothing to exchange
            uid = kernels().rccl_unique_id()
        else:
            key = f"hq_rccl_uid_{next(_uid_counter)}"
            store = dist.distributed_c10d._get_default_store()
            if self.rank == 0:
                store.set(key, kernels().rccl_unique_id())
            uid = store.get(key)        # rank 0 reads its own id back: the same store round trip everywhere
            self.uid_via_store = True
        dev = self.store.device.index if self.store.device.index is not None else torch.cuda.current_device()
        red = kernels().Reducer(self.rank, self.world, bytes(uid), dev)
        logger.info(f"native RCCL reducer up (rank {self.rank}/{self.world}, device {dev})")
        return red

    def _build_buckets(self):
        trainable = {n for n, p in self.model.named_parameters() if p.requires_grad}
        group_has_trainable = {}
        for e in self.store.entries:
            for hf, _, _ in e.views:
                if hf in trainable:
                    group_has_trainable[e.group] = True
        elem = 2 if self.allreduce_dtype == "bf16" else 4
        buckets: List[Tuple[int, int, List[str]]] = []
        for g, s, e in self.store.group_ranges():
            if not group_has_trainable.get(g):
                continue
            # emb_bf16: the embeddings group always travels in a bucket of its own, so no other group is ever
            # all-reduced in bf16 with it, whatever --bucket_cap_mb is
            alone = self.allreduce_dtype == "emb_bf16" and (g == "embeddings" or (buckets and "embeddings" in buckets[-1][2]))
            if buckets and not alone and (buckets[-1][1] == s) and (e - buckets[-1][0]) * elem <= self.bucket_cap:
                bs, _, gs = buckets[-1]
                buckets[-1] = (bs, e, gs + [g])
            else:
                buckets.append((s, e, [g]))
        def bucket_dtype(gs):
            if self.allreduce_dtype == "bf16" or (self.allreduce_dtype == "emb_bf16" and "embeddings" in gs):
                return "bf16"
            return "fp32"
        self.buckets = [Bucket(i, s, e, gs, bucket_dtype(gs)) for i, (s, e, gs) in enumerate(buckets)]
        self.group_to_bucket = {g: b for b in self.buckets for g in b.groups}
        if any(b.dtype == "bf16" for b in self.buckets) and self._native is not None:
            self._scratch = torch.empty(self.store.total, dtype=torch.bfloat16, device=self.store.device)
        logger.info("grad buckets (MiB, dtype): " + ", ".join(
            f"{b.numel * (2 if b.dtype == 'bf16' else 4) / 2**20:.1f} {b.dtype}" for b in self.buckets))

    @property
    def bytes_per_sync(self) -> int:
        """Bytes one synchronising backward all-reduces (every bucket once, at its wire dtype)."""
        return sum(b.numel * (2 if b.dtype == "bf16" else 4) for b in self.buckets)

    def broadcast_parameters(self):
        """Rank 0's weights to everyone (DDP constructor semantics)."""
        m = self.store.master
        if self._native is not None:
            self._native.broadcast(m.data_ptr(), m.numel(), 0, 0, torch.cuda.current_stream().cuda_stream)
            self._native.wait(torch.cuda.current_stream().cuda_stream)
        else:
            dist.broadcast(m, 0, group=self.group)
        self.store.mark_master_dirty()
        self.store.sync_compute()
        self.broadcast_done = True

    # ------------------------------------------------------------------ per step
    @property
    def n_buckets(self) -> int:
        return len(self.buckets)

    @property
    def comm_ranks(self) -> Optional[int]:
        """Ranks the native RCCL communicator spans (``ncclCommCount``); None without one."""
        return int(self._native.comm_count) if self._native is not None else None

    def prepare(self, sync: bool = True):
        self.active = sync and (self.world > 1 or self.force)
        self._norm_ready = False
        for b in self.buckets:
            b.pending = len(b.groups)
            b.launched = False
            b.work = None

    def _on_group_ready(self, group: str):
        if not self.active:
            return
        b = self.group_to_bucket.get(group)
        if b is None:
            return
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    def _launch(self, b: Bucket):
        if b.launched:
            return
        b.launched = True
        view = self.store.grad[b.start:b.end]
        self.stats["buckets_launched"] += 1
        self.stats["bytes"] += b.numel * (2 if b.dtype == "bf16" else 4)
        self._seq_hash = (self._seq_hash * 1_000_003 + b.index * 65_537 + b.numel) & 0x7FFFFFFFFFFFFFFF
        side = getattr(self.model, "grad_side_stream", None)
        if self._native is not None:
            stream = torch.cuda.current_stream().cuda_stream
            if side is not None:  # weight grads computed on the side stream
                self._native.fence_from(side.cuda_stream)
            if self.timing and self._first_ev is None:
                self._native.fence_from(stream)
                self._first_ev = torch.cuda.Event(enable_timing=True)
                self._first_ev.record(self._comm_stream())
            if self.verify:
                part = self._probes.get(b.index)
                if part is None:
                    part = self._probes[b.index] = torch.empty(self._PROBE_PARTS, dtype=torch.float32,
                                                               device=self.store.device)
                self._native.probe_f32(view.data_ptr(), b.numel, part.data_ptr(), self._PROBE_PARTS, stream)
            if b.dtype == "bf16":
                self._native.allreduce_bf16(view.data_ptr(), self._scratch[b.start:b.end].data_ptr(), b.numel, stream)
            else:
                self._native.allreduce_f32(view.data_ptr(), b.numel, stream)
            c0, c1 = self._bucket_chunks[b.index]
            self._native.sq_norm_chunks(self.store.grad.data_ptr(), self._norm_chunks.data_ptr(), c0, c1,
                                        self._norm_parts.data_ptr())
        else:
            if side is not None:
                torch.cuda.current_stream().wait_stream(side)
            backend = dist.get_backend(self.group)
            if backend == "nccl":
                b.work = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
            else:
                b.work = dist.all_reduce(view, group=self.group, async_op=True)

    def finalize(self):
        if not self.active:
            return
        for b in self.buckets:      # groups that never reported (e.g. unused heads): reduce anyway, in order
            if not b.launched:
                self._launch(b)
        if self._native is not None:
            if self.timing:
                cur = torch.cuda.current_stream()
                done_bwd = torch.cuda.Event(enable_timing=True)
                done_bwd.record(cur)
                done_comm = torch.cuda.Event(enable_timing=True)
                done_comm.record(self._comm_stream())
                self._tev.append((self._first_ev, done_bwd, done_comm))
                self._first_ev = None
            self._native.wait(torch.cuda.current_stream().cuda_stream)
            for c0, c1 in self._uncovered:
                kernels().sq_norm_chunks(self.store.grad, self._norm_chunks, c0, c1, self._norm_parts)
            self._norm_ready = True
        else:
            scale = None if dist.get_backend(self.group) == "nccl" else 1.0 / self.world
            for b in self.buckets:
                if b.work is not None:
                    b.work.wait()
                    if scale is not None:
                        self.store.grad[b.start:b.end].mul_(scale)
        self.active = False

    def norm_partials(self) -> Optional[torch.Tensor]:
        """The complete grad-norm partials of the step just finalized (native path), else None (full pass)."""
        return self._norm_parts if self._norm_ready else None

    _PROBE_PARTS = 256

    def _comm_stream(self):
        st = getattr(self, "_ext_stream", None)
        if st is None:
            st = self._ext_stream = torch.cuda.ExternalStream(self._native.comm_stream, device=self.store.device)
        return st

    def pop_timings(self) -> Dict[str, float]:
        """Mean comm span and exposed comm wait (ms) over the steps since the last call (synchronises)."""
        if not self._tev:
            return {}
        torch.cuda.synchronize(self.store.device)
        span = [f.elapsed_time(c) for f, _, c in self._tev if f is not None]
        exposed = [max(0.0, b.elapsed_time(c)) for _, b, c in self._tev]
        self._tev.clear()
        out = {"comm_wait_ms": sum(exposed) / len(exposed)}
        if span:
            out["comm_span_ms"] = sum(span) / len(span)
        return out

    def check_order(self) -> Dict[int, float]:
        """After a synchronised step with ``verify``: {bucket: max |probe − final| / max|final|} — all zeros
        when the comm stream read each bucket only after every kernel writing it had finished (only valid
        while the all-reduce leaves the data unchanged, i.e. a forced world-1 fp32 reducer)."""
        out = {}
        for i, part in self._probes.items():
            b = self.buckets[i]
            ref = kernels().sq_norm_partials(self.store.grad[b.start:b.end], self._PROBE_PARTS)
            torch.cuda.synchronize(self.store.device)
            den = float(ref.abs().max()) or 1.0
            out[i] = float((part - ref).abs().max()) / den
        return out

    def verify_sequence(self):
        """Collective-sequence checker: every rank must have issued the same bucket all-reduces in the
        same order (a divergence is exactly what deadlocks or silently corrupts RCCL/gloo).  The hashes
        travel through the rendezvous TCPStore, not a collective, so a diverged collective stream
        cannot mask the check.  Called by the trainer at epoch end; raises on mismatch."""
        if self.world <= 1:
            return True
        store = dist.distributed_c10d._get_default_store()
        self._verify_calls = getattr(self, "_verify_calls", 0) + 1
        prefix = f"hq_seq/{self._verify_calls}/"
        store.set(prefix + str(self.rank), f"{self._seq_hash}:{self.stats['buckets_launched']}")
        keys = [prefix + str(r) for r in range(self.world)]
        store.wait(keys)
        vals = [store.get(k).decode() for k in keys]
        if len(set(vals)) != 1:
            raise RuntimeError(f"gradient collective sequence diverged across ranks: {vals}")
        return True

    _FP_PARTS = 256

    def take_grad_snapshot(self):
        """Fingerprint of the reduced gradient arena (called by the engine after ``finalize``, before the optimizer
        zeroes it, when ``snapshot_grads`` is set)."""
        g = self.store.grad
        self._grad_fp = fingerprint(g, self._FP_PARTS)
        self._grad_sq = sq_partials(g, self._FP_PARTS)
        self.snapshot_grads = False

    def replica_check(self) -> Dict[str, object]:
        """Data-parallel correctness self-check (a collective: every rank calls it at the same point): all-gathers an
        exact fingerprint of the fp32 master arena — and of the last snapshotted reduced gradient — and compares every
        rank with rank 0.  After a correct DDP step every replica holds bitwise the same weights and gradients; a
        reducer bug (a wrong bucket offset, a bf16 cast-back race, a missed fence) breaks that even when the step
        is fast.  Returns the bench/trainer fields; ``ok`` is False on any mismatch or when the RCCL communicator
        does not span the job."""
        P = self._FP_PARTS
        m = self.store.master
        fm = fingerprint(m, P).cpu()
        sm = sq_partials(m, P)
        has_g = self._grad_fp is not None
        fg = self._grad_fp.cpu() if has_g else torch.zeros(P, dtype=torch.int64)
        sg = self._grad_sq if has_g else torch.zeros(P, dtype=torch.float64)
        local = torch.stack([fm, fg, sm.view(torch.int64), sg.view(torch.int64)])   # [4, P] int64 (f64 bits)
        if dist.is_initialized():
            dev = self.store.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            t = local.to(dev)
            every = [torch.empty_like(t) for _ in range(self.world)]
            dist.all_gather(every, t, group=self.group)
            every = [e.cpu() for e in every]
        else:
            every = [local]
        ref = every[0]
        w_bad = sum(int((e[0] != ref[0]).sum()) for e in every[1:])
        g_bad = sum(int((e[1] != ref[1]).sum()) for e in every[1:])

        def rel(row):
            r0 = ref[row].view(torch.float64)
            den = float(r0.abs().max()) or 1.0
            return max([float((e[row].view(torch.float64) - r0).abs().max()) / den for e in every[1:]] or [0.0])
        comm_ok = self._native is None or self.comm_ranks == self.world
        out = {"weights_equal_across_ranks": w_bad == 0,
               "grads_equal_across_ranks": (g_bad == 0) if has_g else None,
               "replica_mismatch_parts": w_bad + g_bad,
               "max_weight_partial_mismatch": rel(2),
               "max_grad_partial_mismatch": rel(3) if has_g else None,
               "rccl_comm_ranks_ok": comm_ok,
               "replicas_checked": len(every)}
        out["ok"] = bool(w_bad == 0 and g_bad == 0 and comm_ok)
        if not out["ok"]:
            logger.error(f"data-parallel replica check FAILED (rank {self.rank}): {out}")
        return out

    def close(self):
        if self._native is not None:
            self._native.synchronize()
            self._native = None
        if getattr(self, "_set_sched", False):   # back to the single-GPU default (process-wide setting)
            kernels().gemm_set_sched(0)
            self._set_sched = False
        self.model.set_grad_listener(None)
