"""Evaluation callbacks (reference ``modules/model/trainer/callback.py:12-108``).

``SaveBestCallback`` compares with ``operator.gt/lt`` instead of ``eval(f'{a}{op}{b}')``."""
from __future__ import annotations

import logging
import math
import operator

import numpy as np
import torch

from .meters import AverageMeter, MAPMeter

logger = logging.getLogger(__name__)


class TestCallback:
    def at_iteration_end(self, preds, labels, avg_meters):
        self._at_iteration_end(preds, labels, avg_meters)

    def _at_iteration_end(self, *args):
        raise NotImplementedError

    def at_epoch_end(self, avg_meters, trainer):
        self._at_epoch_end(avg_meters, trainer)
        self._reset()

    def _at_epoch_end(self, *args):
        raise NotImplementedError

    def _reset(self):
        pass

    def merge_across_ranks(self):
        """Sharded evaluation: make this rank's state cover every rank's shard (collective; every rank
        calls it before ``at_epoch_end``).  Stateless callbacks have nothing to merge."""


def _acc(true, pred):
    return float((true == pred).float().mean().item())


class AccuracyCallback(TestCallback):
    """Start / end / class accuracy, ignoring ``-1`` span targets."""
    keys = ["start_class", "end_class", "cls"]

    def _at_iteration_end(self, preds, labels, avg_meters):
        s_logit, e_logit, c_logit = (preds[k].detach().float().cpu() for k in self.keys)
        s_true, e_true, c_true = (labels[k].detach().cpu() for k in self.keys)
        s_pred, e_pred, c_pred = (x.argmax(-1) for x in (s_logit, e_logit, c_logit))
        s_ok, e_ok = s_true != -1, e_true != -1
        if s_ok.any():
            avg_meters["s_acc"].update(_acc(s_true[s_ok], s_pred[s_ok]))
        if e_ok.any():
            avg_meters["e_acc"].update(_acc(e_true[e_ok], e_pred[e_ok]))
        avg_meters["c_acc"].update(_acc(c_true, c_pred))

    def _at_epoch_end(self, *args):
        pass


class MAPCallback(TestCallback):
    key = "cls"

    def __init__(self, metric_keys):
        super().__init__()
        self._metric_keys = list(metric_keys)
        self._reset()

    def _at_iteration_end(self, preds, labels, *args):
        probs = torch.softmax(preds[self.key].detach().float().cpu(), dim=-1).numpy()
        self.map_meter.update(keys=self._metric_keys, pred_probas=probs,
                              true_labels=labels[self.key].detach().cpu().numpy())

    def _at_epoch_end(self, avg_meters, *args):
        avg_meters.update(self.map_meter())

    def _reset(self):
        self.map_meter = MAPMeter()

    def merge_across_ranks(self):
        from ..parallel import dist as hqdist
        self.map_meter.merge_states(hqdist.all_gather_object(self.map_meter.state()))


class SaveBestCallback(TestCallback):
    def __init__(self, params):
        super().__init__()
        self.params = params
        self.metric = params.best_metric
        self.best_order = params.best_order
        self._cmp = {">": operator.gt, "<": operator.lt}[self.best_order]
        self.value = 1e10 * (-1 if self.best_order == ">" else 1)

    def _at_iteration_end(self, *args):
        pass

    def _at_epoch_end(self, avg_meters, trainer):
        metrics = {k: v() if isinstance(v, AverageMeter) else v for k, v in avg_meters.items()}
        value = metrics.get(self.metric)
        if value is None or (isinstance(value, float) and math.isnan(value)):
            logger.warning(f"Trainer metrics do not contain metric {self.metric}.")
            return
        if self._cmp(value, self.value):
            self.value = value
            trainer.save_state_dict(self.params.dump_dir / self.params.experiment_name / "best.ch")
            logger.info(f"Best value of {self.metric} was achieved after training step {trainer.global_step} "
                        f"and equals to {self.value:.3f}")
        else:
            logger.info(f"Best value {self.value:.3f} of {self.metric} was not bitten with {value:.3f}")
