"""QA losses (reference ``modules/model/model/loss.py:5-106`` and ``modules/init.py:18-40``).

Differences by design:
* ``WeightedLoss`` keeps per-key losses as *device* tensors (``LossRecord``) instead of calling
  ``.item()`` six times per micro-batch (reference defect D14); the trainer syncs them once per
  logging step.  ``avg_meters`` still receives plain floats when a dict is passed (reference
  behaviour, D13), so callbacks and TensorBoard tags are unchanged.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class LabelSmoothingLossWithLogits(nn.Module):
    """KLDiv(batchmean) against a smoothed one-hot target, or NLL when ``smoothing == 0``."""

    def __init__(self, n_classes: int, *, smoothing: float = 0.0, ignore_index: int = -100):
        super().__init__()
        assert 0.0 <= smoothing <= 1.0
        self.n_classes = n_classes
        self.smoothing = smoothing
        self.confidence = 1.0 - smoothing
        self.ignore_index = ignore_index
        # the ignored class (if it is a real class id) gets no smoothing mass
        self.num_ignore_ixs = 1 + (1 if 0 <= ignore_index < n_classes else 0)

    def forward(self, logits, targets):
        logp = F.log_softmax(logits.float(), dim=-1)
        if self.smoothing <= 0.0:
            return F.nll_loss(logp, targets, ignore_index=self.ignore_index)
        fill = self.smoothing / (self.n_classes - self.num_ignore_ixs)
        with torch.no_grad():
            dist = torch.full((targets.size(0), self.n_classes), fill, device=logits.device, dtype=logp.dtype)
            dist.scatter_(-1, targets.unsqueeze(-1), self.confidence)
            if 0 <= self.ignore_index < self.n_classes:
                dist[:, self.ignore_index] = 0.0
        return F.kl_div(logp, dist, reduction="batchmean")


class BinaryFocalLossWithLogits(nn.Module):
    def __init__(self, alpha: float = 1.0, gamma: float = 2.0):
        super().__init__()
        self.alpha, self.gamma = alpha, gamma

    def forward(self, inputs, targets):
        bce = F.binary_cross_entropy_with_logits(inputs, targets, reduction="none")
        p = torch.exp(-bce)
        return torch.mean(self.alpha * (1.0 - p) ** self.gamma * bce)


class FocalLossWithLogits(nn.Module):
    """NLL over α(1-p)^γ·log p (reference ``loss.py:57-71``)."""

    def __init__(self, alpha: float = 1.0, gamma: float = 2.0, *, ignore_index: int = -1, reduction: str = "mean"):
        super().__init__()
        self.alpha, self.gamma = alpha, gamma
        self.ignore_index, self.reduction = ignore_index, reduction

    def forward(self, inputs, targets):
        logp = F.log_softmax(inputs.float(), dim=-1)
        p = torch.exp(logp)
        return F.nll_loss(self.alpha * (1.0 - p) ** self.gamma * logp, targets, ignore_index=self.ignore_index,
                          reduction=self.reduction)


class LossRecord(dict):
    """Per-key detached device losses of one micro-batch (materialised lazily with one sync)."""

    def to_floats(self) -> Dict[str, float]:
        if not self:
            return {}
        keys = list(self.keys())
        vals = torch.stack([self[k].float().reshape(()) for k in keys]).tolist()
        return dict(zip(keys, vals))


class WeightedLoss:
    """Σ_k w_k · loss_k(pred[k], target[k]) over {start_class, end_class, start_reg, end_reg, cls}."""

    _KEYS = ("start_class", "end_class", "start_reg", "end_reg", "cls")

    def __init__(self, init_losses: Dict[str, Tuple[nn.Module, float]]):
        from .heads import fused_loss_config
        self._losses = init_losses
        self.last: Optional[LossRecord] = None
        # predictions from the fused GPU heads + this exact loss set: one kernel for all five terms
        self._fused_cfg = fused_loss_config(init_losses) if os.environ.get("HQ_FUSED_LOSS", "1") != "0" else None

    def __call__(self, preds, targets, *, avg_meters=None):
        assert set(preds) >= set(self._losses), "missing predictions"
        assert set(targets) >= set(self._losses), "missing targets"
        from .heads import fused_loss, fused_loss_usable
        if fused_loss_usable(preds, self._fused_cfg):
            full, vals = fused_loss(preds, targets, self._fused_cfg)
            rec = LossRecord({k: vals[i] for i, k in enumerate(self._KEYS)})
            rec["loss"] = vals[5]
            self.last = rec
            if avg_meters is not None:
                avg_meters.update(rec.to_floats())
            return full
        lens = targets.get("segment_lengths")
        if lens is not None and len(lens) > 1:
            return self._segmented(preds, targets, lens, avg_meters)
        rec = LossRecord()
        full = 0.0
        for key, (fn, weight) in self._losses.items():
            loss = fn(preds[key].float(), targets[key])
            rec[key] = loss.detach()
            full = full + weight * loss
        rec["loss"] = full.detach()
        self.last = rec
        if avg_meters is not None:
            avg_meters.update(rec.to_floats())
        return full

    def _segmented(self, preds, targets, lens, avg_meters):
        """Merged micro-batches (``data.collate.merge_micro_batches``): each segment is one of the reference's
        micro-batches, scored exactly as the reference scores it — span logits cut to that micro-batch's own
        padded length, every loss module normalising over that segment alone — and the segment losses are
        averaged: the reference's mean of per-micro-batch means (``trainer.py:197-204``).  The CPU oracle of
        the loss kernel's segment mode; the record holds the segment means of every term."""
        S = len(lens)
        B = preds["cls"].shape[0]
        bs = B // S
        assert bs * S == B, "segments must split the batch into equal parts"
        sums: Dict[str, torch.Tensor] = {}
        full = 0.0
        for s, Ls in enumerate(lens):
            rows = slice(s * bs, (s + 1) * bs)
            part = 0.0
            for key, (fn, weight) in self._losses.items():
                p = preds[key][rows]
                if key in ("start_class", "end_class"):
                    p = p[:, :int(Ls)]
                loss = fn(p.float(), targets[key][rows])
                sums[key] = sums[key] + loss.detach() if key in sums else loss.detach()
                part = part + weight * loss
            full = full + part
        full = full / S
        rec = LossRecord({k: v / S for k, v in sums.items()})
        rec["loss"] = full.detach()
        self.last = rec
        if avg_meters is not None:
            avg_meters.update(rec.to_floats())
        return full

    def to(self, device):
        for key in self._losses:
            self._losses[key][0].to(device)
        return self


def build_loss(params, train_weights=None, n_classes: int = 5) -> WeightedLoss:
    """Reference ``init_loss`` (``modules/init.py:18-40``)."""
    def w(name):
        return getattr(params, name, 1)

    label_weights = None if train_weights is None else train_weights.get("label_weights")
    kind = getattr(params, "loss", "ce")
    if kind == "ce":
        cls_loss = nn.CrossEntropyLoss(weight=None if label_weights is None else label_weights.float())
    elif kind == "focal":
        cls_loss = FocalLossWithLogits(alpha=params.focal_alpha, gamma=params.focal_gamma)
    elif kind == "smooth":
        cls_loss = LabelSmoothingLossWithLogits(n_classes=n_classes, smoothing=params.smooth_alpha)
    else:
        raise NotImplementedError(kind)
    return WeightedLoss({"start_class": (nn.CrossEntropyLoss(ignore_index=-1), w("w_start")),
                         "end_class": (nn.CrossEntropyLoss(ignore_index=-1), w("w_end")),
                         "start_reg": (nn.MSELoss(), w("w_start_reg")),
                         "end_reg": (nn.MSELoss(), w("w_end_reg")),
                         "cls": (cls_loss, w("w_cls"))})
