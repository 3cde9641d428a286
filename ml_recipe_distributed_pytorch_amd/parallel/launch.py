"""Process launch plan: one process per GPU (reference ``modules/train.py:18-148`` semantics) or the
torchrun env contract.

Reference contract (no ``RANK`` env): ``--local_rank`` is the NODE rank, ``--dist_world_size`` the
number of nodes; every node spawns one worker per local GPU and worker ``i`` on node ``n`` gets global
rank ``n·gpus_per_node + i``.  Fixes: D3 (device = LOCAL GPU index), D4 (torchrun env wins, no
double spawning), D5 (a 1-process run needs no process group and never calls collectives), D20
(``n_jobs`` clamp never reaches 0).  CPU runs may spawn several gloo ranks (``--nproc_per_node``)
to rehearse multi-node on one host.
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from typing import Callable, Optional

import torch

logger = logging.getLogger(__name__)


@dataclass
class LaunchPlan:
    node_rank: int           # reference --local_rank (node index), -1 = not distributed
    n_nodes: int
    nproc_per_node: int
    use_gpu: bool
    backend: str
    init_method: str
    env: bool = False        # torchrun-style env launch (RANK/WORLD_SIZE set)

    @property
    def world_size(self) -> int:
        if self.env:
            return int(os.environ["WORLD_SIZE"])
        return self.n_nodes * self.nproc_per_node

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def spawn(self) -> bool:
        return not self.env and self.nproc_per_node > 1

    def global_rank(self, local_idx: int) -> int:
        if self.env:
            return int(os.environ["RANK"])
        return max(self.node_rank, 0) * self.nproc_per_node + local_idx


def make_plan(params) -> LaunchPlan:
    env = "RANK" in os.environ and "WORLD_SIZE" in os.environ
    use_gpu = bool(getattr(params, "gpu", False)) and torch.cuda.is_available()
    ngpu = torch.cuda.device_count() if use_gpu else 0
    nproc = params.nproc_per_node if getattr(params, "nproc_per_node", None) else (ngpu or 1)
    if use_gpu and nproc > ngpu:
        raise ValueError(f"--nproc_per_node {nproc} exceeds the {ngpu} visible GPUs.")
    backend = params.dist_backend if use_gpu else "gloo"
    plan = LaunchPlan(node_rank=params.local_rank, n_nodes=max(1, params.dist_world_size), nproc_per_node=nproc,
                      use_gpu=use_gpu, backend=backend, init_method=params.dist_init_method, env=env)
    if plan.distributed and not plan.env and plan.node_rank == -1:
        raise AttributeError("Specify local rank.")
    return plan


def clamp_jobs(n_jobs: int, nproc_per_node: int) -> int:
    cpus = os.cpu_count() or 1
    n = min(n_jobs, max(1, cpus // 2))
    if nproc_per_node * n > cpus:
        n = max(1, cpus // (2 * nproc_per_node))
    return n


def launch(worker: Callable, plan: LaunchPlan, *args):
    """Run ``worker(local_idx, plan, *args)`` in this process or in ``nproc_per_node`` spawned ones."""
    if plan.spawn:
        import torch.multiprocessing as mp
        if plan.distributed:
            logger.warning("It can take a while to start all worker processes and connect to the master host.")
        mp.spawn(worker, nprocs=plan.nproc_per_node, args=(plan,) + args, join=True)
    else:
        local = int(os.environ.get("LOCAL_RANK", "0")) if plan.env else 0
        worker(local, plan, *args)


def device_for(plan: LaunchPlan, local_idx: int) -> torch.device:
    if plan.use_gpu:
        return torch.device("cuda", local_idx)
    return torch.device("cpu")
