"""Trainer (placeholder: filled in below)."""
from __future__ import annotations

from ..models.params import no_decay


def optimizer_groups(named_params, weight_decay: float):
    """Reference ``_get_optimized_parameters`` param groups (``modules/init.py:125-131``)."""
    named = list(named_params)
    return [{"params": [p for n, p in named if not no_decay(n)], "weight_decay": weight_decay},
            {"params": [p for n, p in named if no_decay(n)], "weight_decay": 0.0}]
