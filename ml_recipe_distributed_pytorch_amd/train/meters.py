"""Metric meters (reference ``modules/model/trainer/meters.py:10-56``)."""
from __future__ import annotations

from collections import defaultdict

import numpy as np


class AverageMeter:
    """Running mean of ``update(value)`` calls; calling the meter returns the mean."""

    def __init__(self):
        self._counter = 0
        self._avg_value = 0.0

    def __call__(self):
        return self._avg_value

    def update(self, value):
        self._counter += 1
        self._avg_value += (float(value) - self._avg_value) / self._counter

    @property
    def count(self) -> int:
        return self._counter

    @property
    def sum(self) -> float:
        return self._avg_value * self._counter

    @classmethod
    def from_sum_count(cls, total: float, count: int) -> "AverageMeter":
        """A meter whose mean is ``total / count`` (merging per-rank meters of a sharded evaluation)."""
        m = cls()
        m._counter = int(count)
        m._avg_value = float(total) / count if count else 0.0
        return m


class APMeter:
    """Average precision of one binary target (sklearn ``average_precision_score``)."""

    def __init__(self):
        self.reset()

    def __call__(self):
        from sklearn import metrics
        y_true = np.asarray(self.true_labels)
        if y_true.size == 0 or not y_true.any():
            return float("nan")
        return float(metrics.average_precision_score(y_true, np.asarray(self.pred_probas)))

    def update(self, pred_probas, true_labels):
        self.pred_probas.extend(np.asarray(pred_probas).tolist())
        self.true_labels.extend(np.asarray(true_labels).tolist())

    def reset(self):
        self.pred_probas = []
        self.true_labels = []

    def extend(self, other: "APMeter"):
        self.pred_probas.extend(other.pred_probas)
        self.true_labels.extend(other.true_labels)


class MAPMeter:
    """Per-class AP dict plus their mean under ``'map'``."""

    def __init__(self):
        self.reset()

    def __call__(self):
        out = {k: v() for k, v in self.aps_dict.items()}
        vals = [v for v in out.values() if v == v]
        out["map"] = float(np.mean(vals)) if vals else float("nan")
        return out

    def update(self, keys, pred_probas, true_labels):
        assert len(keys) == pred_probas.shape[-1]
        for i, key in enumerate(keys):
            self.aps_dict[key].update(pred_probas[:, i], true_labels == i)

    def reset(self):
        self.aps_dict = defaultdict(APMeter)

    def state(self):
        """Plain lists (picklable) of every class' predictions and targets."""
        return {k: (list(v.pred_probas), list(v.true_labels)) for k, v in self.aps_dict.items()}

    def merge_states(self, states):
        """Rebuild from the ``state()`` of every shard, in rank order (the union of the shards)."""
        self.reset()
        for st in states:
            for k, (p, t) in st.items():
                self.aps_dict[k].pred_probas.extend(p)
                self.aps_dict[k].true_labels.extend(t)
