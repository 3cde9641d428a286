"""Trainer: epochs, evaluation, checkpoints, TensorBoard (reference ``modules/model/trainer/trainer.py:48-403``).

Same constructor fields, the same ``train(after_epoch_funcs)`` / ``test(epoch, callbacks)`` /
``save_state_dict`` / ``load_state_dict`` API and the same checkpoint keys, with these deliberate
differences:

* the hot loop is ``TrainEngine`` (fused encoder, arena gradients, on-device clip, fused AdamW);
* data parallelism is ``GradReducer`` over RCCL instead of DDP; micro-batch accumulation does not
  all-reduce (D1); evaluation runs on the unwrapped model (D2) — rank 0 only, or sharded over
  ranks with ``eval_shard``;
* ``DistributedSampler.set_epoch`` is called every epoch (D6);
* checkpoints save under ``'apex'`` never, load tolerates ``'apex'``/``'amp'`` (D7) and also
  store/restore ``epoch`` + ``epoch_complete``: resuming an end-of-epoch checkpoint continues at the
  next epoch; resuming ``interrupt.ch`` (written mid-epoch) re-enters the interrupted epoch and skips
  the micro-batches that epoch had already consumed (same sampler permutation under a fixed seed);
* apex levels map to native bf16 mixed precision (O0 → fp32 compute);
* per-step losses stay on device; one device→host sync per ``log_every`` optimizer steps (D14);
* ``perf/samples_per_sec`` and ``perf/step_ms`` TensorBoard scalars.
"""
from __future__ import annotations

import functools
import logging
import os
import shutil
import time
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Optional

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, DistributedSampler, RandomSampler, WeightedRandomSampler

from ..models.params import no_decay
from ..parallel import dist as hqdist
from ..parallel.reducer import GradReducer
from ..utils.tb import SummaryWriter
from .callbacks import TestCallback
from .amp import apex_to_precision, resolve_precision  # noqa: F401  (apex_to_precision re-exported)
from .engine import TrainEngine, prefetch_to_device, to_device
from .meters import AverageMeter
from .optim import get_linear_schedule_with_warmup

logger = logging.getLogger(__name__)


def optimizer_groups(named_params, weight_decay: float):
    """Reference ``_get_optimized_parameters`` param groups (``modules/init.py:125-131``)."""
    named = list(named_params)
    return [{"params": [p for n, p in named if not no_decay(n)], "weight_decay": weight_decay},
            {"params": [p for n, p in named if no_decay(n)], "weight_decay": 0.0}]


def time_profiler(fun):
    @functools.wraps(fun)
    def wrapped(*args, **kwargs):
        start = time.perf_counter()
        try:
            return fun(*args, **kwargs)
        finally:
            logger.info(f"Execution of {fun.__name__} took {time.perf_counter() - start:.3f} sec.")
    return wrapped


def _fault_hook(rank: int, step: int):
    """Test-only fault injection: ``HQ_FAULT=rank:step:kind`` (kind = interrupt | error)."""
    spec = os.environ.get("HQ_FAULT")
    if not spec:
        return
    r, s, kind = spec.split(":")
    if int(r) == rank and int(s) == step:
        if kind == "interrupt":
            raise KeyboardInterrupt(f"injected at step {step}")
        raise RuntimeError(f"injected fault at step {step}")


class EvalShardSampler(torch.utils.data.Sampler):
    """Rank ``r`` of ``w`` evaluates indices ``r, r + w, …`` — no padding duplicates (unlike
    ``DistributedSampler``), so the union of the shards is exactly the test set."""

    def __init__(self, n: int, rank: int, world: int):
        self.idx = list(range(rank, n, world))

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


@dataclass
class Trainer:
    model: Any
    loss: Any
    collate_fun: Any
    optimizer: Any = None
    train_dataset: Any = None
    test_dataset: Any = None
    writer_dir: Any = None
    device: Any = torch.device("cpu")
    local_rank: int = -1
    gpu_id: Optional[int] = None
    sync_bn: bool = False
    n_epochs: int = 0
    train_batch_size: int = 32
    test_batch_size: int = 32
    batch_split: int = 1
    n_jobs: int = 4
    warmup_coef: float = 0.01
    max_grad_norm: float = 1.0
    apex_level: Optional[str] = None
    apex_verbosity: int = 1
    apex_loss_scale: Optional[float] = None
    train_weights: Any = None
    drop_optimizer: bool = False
    debug: bool = False
    # --- MI355X additions ---
    bucket_cap_mb: float = 32.0
    allreduce_dtype: str = "fp32"
    no_sync_accum: bool = True
    log_every: int = 1
    profile: bool = False
    cuda_graph: bool = False
    eval_shard: bool = False
    precision: Optional[str] = None
    torch_profile_dir: Optional[str] = None
    torch_profile_steps: str = "3:5"
    sampler_seed: int = 0   # per-epoch sampler permutation = f(sampler_seed, epoch): reproducible on resume
    merge_segments: int = 1  # micro-batches per merged forward/backward pass (exact-objective merge, engine.py)
    extra_state: dict = field(default_factory=dict)

    def __post_init__(self):
        self.device = torch.device(self.device)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        if self.sync_bn and self.local_rank != -1:
            logger.info("sync_bn: the BERT encoder has no BatchNorm layers; nothing to convert.")
        prec = resolve_precision(self.precision, self.apex_level, self.device, self.apex_loss_scale)
        if hasattr(self.model, "set_precision"):
            self.model.set_precision(prec)
        self.model = self.model.to(self.device)
        self.loss = self.loss.to(self.device)
        self.train_sampler = self._init_train_sampler()
        self.train_dataloader = self._init_dataloader(self.train_dataset, "Train",
                                                      batch_size=int(self.train_batch_size // self.batch_split),
                                                      sampler=self.train_sampler, drop_last=True)
        test_sampler = None
        if self.test_dataset is not None and self.eval_shard and self.world > 1:
            test_sampler = EvalShardSampler(len(self.test_dataset), self.rank, self.world)
        self.test_dataloader = self._init_dataloader(self.test_dataset, "Test", batch_size=self.test_batch_size,
                                                     sampler=test_sampler, drop_last=False)
        self.scheduler = None
        if self.train_dataloader is not None and self.optimizer is not None and self.warmup_coef > 0:
            num_training_steps = self.n_epochs * len(self.train_dataloader) // self.batch_split
            num_warmup_steps = int(num_training_steps * self.warmup_coef)
            logger.info(f"Warmup schedule is used. #Training steps: {num_training_steps}. "
                        f"#Warmup steps: {num_warmup_steps}.")
            self.scheduler = get_linear_schedule_with_warmup(self.optimizer, num_warmup_steps, num_training_steps)
        logger.info(f"Precision: {prec} (apex_level {self.apex_level} mapped to native mixed precision).")
        self.reducer = None
        if self.world > 1 and self.optimizer is not None:
            self.reducer = GradReducer(self.model, bucket_cap_mb=self.bucket_cap_mb,
                                       allreduce_dtype=self.allreduce_dtype)
        self.engine = None
        if self.optimizer is not None:
            G = max(1, int(self.merge_segments))
            if self.batch_split % G:
                raise ValueError(f"merge_segments {G} must divide batch_split {self.batch_split}")
            self.engine = TrainEngine(self.model, self.loss, self.optimizer, scheduler=self.scheduler,
                                      reducer=self.reducer, max_grad_norm=self.max_grad_norm,
                                      batch_split=self.batch_split // G, no_sync_accum=self.no_sync_accum,
                                      profile=self.profile, graph=self.cuda_graph, merge_segments=G)
        self.global_step = 0
        self.start_epoch = 1
        self.epoch_complete = True
        self._resume_skip = 0  # micro-batches of the resumed (interrupted) epoch already consumed
        self.writer = self._init_writer(self.local_rank, self.writer_dir) if self.rank == 0 else None
        if self.debug:
            self.n_epochs = 2  # after the scheduler was built, as the reference (D8)

    # ------------------------------------------------------------------ setup helpers
    def _init_train_sampler(self):
        """Every sampler draws its epoch permutation from (sampler_seed, epoch) alone — DistributedSampler via
        seed + set_epoch, the world-1 samplers via their own torch.Generator re-seeded at each epoch start — so
        a run resumed from interrupt.ch replays the interrupted epoch's permutation exactly (the global RNG,
        which dropout seeds consume, is not part of it)."""
        if self.train_dataset is None:
            return None
        self._sampler_gen = torch.Generator()
        if self.world > 1:
            sampler = DistributedSampler(self.train_dataset, seed=int(self.sampler_seed))
        elif self.train_weights is not None and self.train_weights.get("sampler_weights") is not None:
            w = self.train_weights["sampler_weights"]
            assert len(w) == len(self.train_dataset)
            sampler = WeightedRandomSampler(w, len(self.train_dataset), generator=self._sampler_gen)
        else:
            sampler = RandomSampler(self.train_dataset, generator=self._sampler_gen)
        logger.info(f"Used train sampler: {type(sampler).__name__}.")
        return sampler

    def _seed_sampler(self, epoch_i: int):
        if isinstance(self.train_sampler, DistributedSampler):
            self.train_sampler.set_epoch(epoch_i)  # reference never did (D6)
        elif self.train_sampler is not None:
            self._sampler_gen.manual_seed(int(self.sampler_seed) * 1_000_003 + int(epoch_i))

    def epoch_indices(self, epoch_i: int):
        """The sample order of epoch ``epoch_i`` on this rank (re-seeds the sampler, as _train does)."""
        self._seed_sampler(epoch_i)
        return list(iter(self.train_sampler))

    def _init_dataloader(self, dataset, name, *, batch_size=1, sampler=None, drop_last=False):
        if dataset is None:
            return None
        logger.info(f"{name} dataset len: {len(dataset)}. #JOBS: {self.n_jobs}.")
        return DataLoader(dataset, batch_size=batch_size, num_workers=self.n_jobs, sampler=sampler,
                          drop_last=drop_last, shuffle=False, collate_fn=self.collate_fun,
                          pin_memory=self.device.type == "cuda", persistent_workers=False)

    @staticmethod
    def _init_writer(local_rank, writer_dir):
        if writer_dir is None or local_rank not in (-1, 0):
            return None
        logger.warning(f"Directory {writer_dir} will be cleaned before SummaryWriter initialization. "
                       f"To prevent missing important information, use different experiment names.")
        shutil.rmtree(writer_dir, ignore_errors=True)
        return SummaryWriter(log_dir=writer_dir)

    def _get_lr(self):
        return self.optimizer.param_groups[0]["lr"]

    @staticmethod
    def _console_str(values):
        return ", ".join(f"{k}: {(v() if isinstance(v, AverageMeter) else v):.3e}" for k, v in values.items())

    def _update_writer(self, values, *, prefix):
        if self.writer is None:
            return
        for k, v in values.items():
            self.writer.add_scalar(f"{prefix}/{k}", v() if isinstance(v, AverageMeter) else v,
                                   global_step=self.global_step)

    def set_train(self):
        mods = getattr(self.model, "list_of_trainable_modules", None)
        if self.apex_level is None and mods:
            for m in mods:
                m.train()
        else:
            self.model.train()

    def set_eval(self):
        self.model.eval()

    def _to_device(self, data):
        return to_device(data, self.device)

    # ------------------------------------------------------------------ training
    def train(self, after_epoch_funcs=None):
        if self.train_dataloader is None:
            logger.warning("You have not specified train dataset, so you cannot run train method.")
            return
        after_epoch_funcs = after_epoch_funcs or []
        for epoch_i in range(self.start_epoch, self.n_epochs + 1):
            self.epoch = epoch_i
            self.epoch_complete = False
            self._train(epoch_i)
            self.epoch_complete = True
            if self.reducer is not None:
                self.reducer.verify_sequence()
                rep = self.reducer.replica_check()   # every replica must hold bitwise rank 0's weights
                if not rep["ok"]:
                    raise RuntimeError(f"data-parallel replicas diverged at the end of epoch {epoch_i}: {rep}")
            for func in after_epoch_funcs:
                func(epoch_i)

    @time_profiler
    def _train(self, epoch_i):
        from tqdm.auto import tqdm
        self.set_train()
        self.optimizer.zero_grad()
        self._seed_sampler(epoch_i)
        self.engine.micro = 0
        self.engine._pending = []
        avg = {}
        last_t, last_step = time.perf_counter(), self.global_step
        samples_per_step = self.train_batch_size * self.world
        steady = [0, 0.0]  # optimizer steps and seconds after the first two logged intervals (warm-up)
        logged = 0
        loader, skip = self.train_dataloader, self._resume_skip
        self._resume_skip = 0
        if skip:
            # re-enter an interrupted epoch: drop the samples it had consumed (whole optimizer steps)
            micro_bs = int(self.train_batch_size // self.batch_split)
            rest = self.epoch_indices(epoch_i)[skip * micro_bs:]
            logger.info(f"Resuming epoch {epoch_i} after {skip} consumed micro-batches ({len(rest)} samples left).")
            loader = DataLoader(self.train_dataset, batch_size=micro_bs, num_workers=self.n_jobs, sampler=rest,
                                drop_last=True, shuffle=False, collate_fn=self.collate_fun,
                                pin_memory=self.device.type == "cuda")
        self._epoch_start_step = self.global_step - skip // max(1, self.batch_split)
        # HQ_TRACE_SAMPLES=<file> (tests): append each consumed micro-batch's sample indices as a JSON line
        trace = os.environ.get("HQ_TRACE_SAMPLES")
        if trace:
            order = self.epoch_indices(epoch_i)
            self._seed_sampler(epoch_i)   # the loader draws the same permutation again
            trace_mb = int(self.train_batch_size // self.batch_split)
        data = tqdm(loader, desc=f"Train (epoch #{epoch_i} / {self.n_epochs})",
                    disable=self.rank != 0 or not logger.isEnabledFor(logging.INFO))
        # each micro-batch's host → device copy runs on a copy stream under the previous micro-step (DevicePrefetcher)
        for i, (inputs, labels) in enumerate(prefetch_to_device(data, self.device)):
            if trace:
                import json
                with open(trace, "a") as f:
                    f.write(json.dumps({"epoch": epoch_i, "rank": self.rank,
                                        "idx": [int(x) for x in order[(skip + i) * trace_mb:(skip + i + 1) * trace_mb]]})
                            + "\n")
            res = self.engine.micro_step(inputs, labels)
            if res is None:
                continue
            self.global_step += 1
            self._torch_profiler_step()
            _fault_hook(self.rank, self.global_step)
            if self.global_step % max(1, self.log_every) == 0 or self.debug:
                avg = res.losses.to_floats()  # the one device→host sync per log step
                avg["lr"] = res.lr
                now = time.perf_counter()
                steps = self.global_step - last_step
                if steps > 0:
                    avg["perf/samples_per_sec"] = samples_per_step * steps / max(now - last_t, 1e-9)
                    avg["perf/step_ms"] = (now - last_t) / steps * 1e3
                    logged += 1
                    if logged > 2:
                        steady[0] += steps
                        steady[1] += now - last_t
                last_t, last_step = now, self.global_step
                tb = {k: v for k, v in avg.items() if not k.startswith("perf/")}
                self._update_writer(tb, prefix="train")
                if self.writer is not None:
                    for k in ("perf/samples_per_sec", "perf/step_ms"):
                        if k in avg:
                            self.writer.add_scalar(k, avg[k], global_step=self.global_step)
                    if self.profile:
                        for k, v in res.timings.items():
                            self.writer.add_scalar(f"perf/{k}", v, global_step=self.global_step)
                        if "comm_wait_ms" in res.timings:  # SURVEY §5.5 tag name
                            self.writer.add_scalar("perf/comm_ms", res.timings["comm_wait_ms"],
                                                   global_step=self.global_step)
                data.set_postfix_str(self._console_str({k: v for k, v in avg.items() if not k.startswith("perf")}))
            if self.debug:
                logger.info("Training was interrupted because of debug mode.")
                break
        if steady[0] > 0 and self.rank == 0:  # comparable with bench.py's samples/s (same step, host clock)
            logger.info(f"Train throughput (epoch {epoch_i}, {steady[0]} steady-state steps): "
                        f"{samples_per_step * steady[0] / steady[1]:.1f} samples/sec, "
                        f"{steady[1] / steady[0] * 1e3:.2f} ms/step.")

    # ------------------------------------------------------------------ torch.profiler export
    def _torch_profiler_step(self):
        """SURVEY §5.1 optional torch.profiler trace: optimizer steps ``first..last`` (1-based) of this
        run are captured with CPU + HIP activities and written as a Chrome trace per rank."""
        if not self.torch_profile_dir:
            return
        first, last = (int(x) for x in str(self.torch_profile_steps).split(":"))
        prof = getattr(self, "_tprof", None)
        if prof is False:
            return
        if prof is None and first - 1 <= self.global_step < last:  # armed after step first-1 (>= step 1)
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._tprof = torch.profiler.profile(activities=acts, record_shapes=True)
            self._tprof.__enter__()
        elif prof is not None and self.global_step >= last:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            prof.__exit__(None, None, None)
            os.makedirs(self.torch_profile_dir, exist_ok=True)
            path = os.path.join(self.torch_profile_dir, f"trace_rank{self.rank}_steps{first}-{last}.json")
            prof.export_chrome_trace(path)
            logger.info(f"torch.profiler trace written to {path}")
            self._tprof = False  # done; never re-arm

    # ------------------------------------------------------------------ evaluation
    def test(self, epoch_i, *, callbacks=None):
        sharded = self.eval_shard and self.world > 1
        if self.rank == 0 or sharded:
            if self.test_dataloader is None:
                logger.warning("You have not specified test dataset, so you cannot run test method.")
            else:
                callbacks = list(callbacks or [])
                assert all(isinstance(c, TestCallback) for c in callbacks)
                with torch.no_grad():
                    self._test(epoch_i, callbacks=callbacks)
        if self.world > 1:
            logger.warning("Waiting till validation ends in main process..")
            hqdist.barrier()

    @time_profiler
    @torch.no_grad()
    def _test(self, epoch_i, *, callbacks=None):
        from tqdm.auto import tqdm
        self.set_eval()
        avg_meters = defaultdict(AverageMeter)
        data = tqdm(self.test_dataloader, desc=f"Test (epoch #{epoch_i} / {self.n_epochs})",
                    disable=self.rank != 0 or not logger.isEnabledFor(logging.INFO))
        for i, batch in enumerate(data):
            inputs, labels = self._to_device((batch[0], batch[1]))
            preds = self.model(**inputs)
            self.loss(preds, labels)
            for k, v in self.loss.last.to_floats().items():
                avg_meters[k].update(v)
            for cb in callbacks or []:
                cb.at_iteration_end(preds, labels, avg_meters)
            if self.debug and i >= 10:
                logger.info("Test was interrupted because of debug mode.")
                break
        if self.eval_shard and self.world > 1:
            self._merge_eval_shards(avg_meters, callbacks or [])
        for cb in callbacks or []:
            cb.at_epoch_end(avg_meters, self)
        self._update_writer(avg_meters, prefix="test")
        metrics = {k: v() if isinstance(v, AverageMeter) else v for k, v in avg_meters.items()}
        logger.info(f"Test metrics after epoch {epoch_i} - {self._console_str(metrics)}")
        self.last_metrics = metrics
        self.set_train()

    @staticmethod
    def _merge_eval_shards(avg_meters, callbacks):
        """Collective: every rank ends with the meters of the whole test set.  Keys are the union over
        ranks (a shard may lack e.g. ``s_acc`` when none of its spans is valid), reduced as fixed-order
        (sum, count) pairs; callbacks merge their own state (MAP: gathered predictions)."""
        keys = sorted(set().union(*hqdist.all_gather_object(sorted(avg_meters))))
        local = [avg_meters[k] if k in avg_meters else AverageMeter() for k in keys]
        red = hqdist.all_reduce_sum_floats([m.sum for m in local] + [float(m.count) for m in local])
        n = len(keys)
        for i, k in enumerate(keys):
            avg_meters[k] = AverageMeter.from_sum_count(red[i], int(red[n + i]))
        for cb in callbacks:
            cb.merge_across_ranks()

    # ------------------------------------------------------------------ checkpoints
    def _unwrapped(self):
        return getattr(self.model, "module", self.model)

    def state_dict(self):
        return {"model": self._unwrapped().state_dict(),
                "optimizer": self.optimizer.state_dict() if self.optimizer is not None else None,
                "scheduler": self.scheduler.state_dict() if self.scheduler is not None else None,
                "global_step": self.global_step,
                "epoch": getattr(self, "epoch", 0),
                "epoch_complete": bool(self.epoch_complete),
                "epoch_start_step": int(getattr(self, "_epoch_start_step", self.global_step)),
                **self.extra_state}

    def save_state_dict(self, path_):
        if self.rank != 0:
            return
        if self.debug:
            logger.info(f"Model was not saved to {path_} because of debug mode.")
            return
        tmp = str(path_) + ".tmp"
        torch.save(self.state_dict(), tmp)
        os.replace(tmp, path_)
        logger.info(f"State dict was saved to {path_}.")

    def load_state_dict(self, path_):
        if not os.path.exists(path_):
            logger.warning(f"Checkpoint {path_} does not exist, so checkpoint was not loaded.")
            return
        state = torch.load(path_, map_location="cpu", weights_only=True)
        self._unwrapped().load_state_dict(state["model"])
        self.global_step = int(state.get("global_step", 0))
        if "epoch" in state and state["epoch"]:
            if state.get("epoch_complete", True):
                self.start_epoch = int(state["epoch"]) + 1
            else:  # interrupt.ch: finish the interrupted epoch instead of skipping its remainder
                self.start_epoch = int(state["epoch"])
                done = self.global_step - int(state.get("epoch_start_step", self.global_step))
                self._resume_skip = max(0, done) * self.batch_split
        logger.info(f"Model weights were loaded from {path_} checkpoint.")
        if not self.drop_optimizer:
            if self.optimizer is not None and state.get("optimizer") is not None:
                self.optimizer.load_state_dict(state["optimizer"])
            if self.scheduler is not None and state.get("scheduler") is not None:
                self.scheduler.load_state_dict(state["scheduler"])
                # the restored optimizer carries the OLD run's last LR: re-evaluate this run's schedule at
                # the restored step so the first resumed step already follows it
                sch = self.scheduler
                for g, base, fn in zip(self.optimizer.param_groups, sch.base_lrs, sch.lr_lambdas):
                    g["lr"] = base * fn(sch.last_epoch)
                sch._last_lr = [g["lr"] for g in self.optimizer.param_groups]
            if "apex" in state or "amp" in state:
                logger.info("Checkpoint carries apex AMP state; native bf16 mixed precision needs none (ignored).")
            logger.info(f"Optimizer and scheduler also were restored from {path_} checkpoint.")
        if self.reducer is not None:
            self.reducer.broadcast_parameters()
