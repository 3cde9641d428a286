"""Multi-process loader for datasets whose items are LISTS of chunks (reference
``modules/model/utils/list_dataloader.py:9-97``).

Workers (forked, each holding the dataset once via the pool initializer — no per-task pickling
of the dataset) expand document indices into chunk lists; the parent flattens them into fixed-size
batches and collates.  Differences from the reference, fixing D19:

* results are consumed with ``imap_unordered`` so a worker exception is re-raised in the parent
  (the reference's error callback raised inside the pool thread and the main loop hung on
  ``queue.get()``);
* every wait has a timeout (``timeout_s``) → ``TimeoutError`` instead of a silent hang;
* the pool is always terminated (context-managed generator), ``n_jobs=0`` iterates in-process.
Order is shuffled when ``shuffle`` (reference default in the predictor).
"""
from __future__ import annotations

import logging
import multiprocessing as mp
from typing import Callable, Optional

import numpy as np

logger = logging.getLogger(__name__)

_DATASET = None


def _init_worker(dataset):
    global _DATASET
    _DATASET = dataset


def _expand(idxs):
    return [chunk for i in idxs for chunk in _DATASET[int(i)]]


class ListDataloader:
    def __init__(self, dataset, batch_size: int, *, n_jobs: int = 4, collate_fun: Optional[Callable] = None,
                 buffer_size: int = 1024, shuffle: bool = False, docs_per_task: int = 4, timeout_s: float = 600.0,
                 seed: Optional[int] = None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.collate_fun = collate_fun
        self.n_jobs = max(0, int(n_jobs))
        self.buffer_size = buffer_size
        self.shuffle = shuffle
        self.docs_per_task = max(1, docs_per_task)
        self.timeout_s = timeout_s
        self.seed = seed

    def process_batch(self, batch):
        return self.collate_fun(batch) if self.collate_fun is not None else batch

    def _tasks(self):
        idxs = np.arange(len(self.dataset))
        if self.shuffle:
            rng = np.random.default_rng(self.seed) if self.seed is not None else np.random
            rng.shuffle(idxs)
        return [idxs[i:i + self.docs_per_task] for i in range(0, len(idxs), self.docs_per_task)]

    def _chunk_lists(self):
        tasks = self._tasks()
        if self.n_jobs == 0:
            for t in tasks:
                yield [c for i in t for c in self.dataset[int(i)]]
            return
        ctx = mp.get_context("fork")
        pool = ctx.Pool(self.n_jobs, initializer=_init_worker, initargs=(self.dataset,))
        try:
            it = pool.imap_unordered(_expand, tasks, chunksize=1)
            for _ in range(len(tasks)):
                yield it.next(timeout=self.timeout_s)
        except mp.TimeoutError as e:
            raise TimeoutError(f"ListDataloader: no chunk produced within {self.timeout_s}s") from e
        finally:
            pool.terminate()
            pool.join()

    def __iter__(self):
        batch = []
        for chunks in self._chunk_lists():
            for c in chunks:
                batch.append(c)
                if len(batch) == self.batch_size:
                    yield self.process_batch(batch)
                    batch = []
        if batch:
            yield self.process_batch(batch)
