"""Process-group bootstrap and rank helpers.

Backend ``nccl`` is RCCL on ROCm (xGMI inside a node); ``gloo`` is the CPU path (BASELINE config #1
and every multi-process CPU test).  Supports both launch contracts:

* reference: ``--local_rank <node_rank> --dist_world_size <nodes> --dist_init_method tcp://…`` with one
  process per local GPU spawned by ``launch.spawn_workers`` (``modules/train.py:18-148``; D3/D4/D5 fixed);
* torchrun / ``torch.distributed.run``: ``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``MASTER_ADDR/PORT``.
"""
from __future__ import annotations

import datetime
import logging
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "gloo"
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_INFO = DistInfo()


def info() -> DistInfo:
    return _INFO


def env_launched() -> bool:
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ


def init_distributed(backend: str, *, init_method: Optional[str] = None, world_size: int = 1, rank: int = 0,
                     local_rank: int = 0, timeout_s: float = 1800.0, use_gpu: bool = True) -> DistInfo:
    """Initialise the default process group (also for world_size == 1: fixes D5) and pick the device."""
    global _INFO
    if env_launched():
        rank = int(os.environ["RANK"])
        world_size = int(os.environ["WORLD_SIZE"])
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        init_method = "env://"
    gpu = use_gpu and torch.cuda.is_available()
    if backend == "nccl" and not gpu:
        logger.warning("nccl (RCCL) backend requested without a GPU: falling back to gloo.")
        backend = "gloo"
    if gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)   # local index (reference D3 used the global rank)
    else:
        device = torch.device("cpu")
    # surface RCCL failures as exceptions instead of hangs
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if not dist.is_initialized():
        kw = dict(backend=backend, init_method=init_method, world_size=world_size, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl" and gpu:
            kw["device_id"] = device
        try:
            dist.init_process_group(**kw)
        except TypeError:
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    _INFO = DistInfo(rank=rank, world_size=world_size, local_rank=local_rank, backend=backend, device=device)
    return _INFO


def barrier():
    """Barrier over the default group (also a 1-rank group: the world-1 rehearsal of the N-rank path)."""
    if dist.is_initialized():
        if _INFO.backend == "nccl" and _INFO.device.type == "cuda":
            dist.barrier(device_ids=[_INFO.device.index])
        else:
            dist.barrier()


def destroy():
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:  # pragma: no cover
            pass


def all_reduce_mean_floats(values, device=None):
    """Average a list of python floats over ranks (used for sharded eval metrics)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return list(values)
    dev = device or _INFO.device
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return (t / dist.get_world_size()).tolist()


def all_gather_object(obj):
    """Every rank's ``obj`` in rank order (``[obj]`` without a process group)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def all_reduce_sum_floats(values, device=None):
    """Element-wise sum of a list of python floats over ranks (float64)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return list(values)
    dev = device or _INFO.device
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.tolist()
