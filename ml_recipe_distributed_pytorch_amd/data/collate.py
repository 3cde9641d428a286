"""Batch collation (reference ``split_dataset.py:480-520``), vectorised.

* ``input_ids`` int64 [b, L] padded with ``pad_token_id`` to the batch max length;
* ``token_type_ids``: BERT → 0 up to and including the first ``[SEP]``, 1 after (and 1 on padding,
  as the reference); RoBERTa → all 0;
* ``attention_mask`` = ``input_ids > 0`` (bool) — reference semantics (for RoBERTa, pad=1 is > 0);
* labels: ``start_class``/``end_class`` int64 (-1 = ignore), ``start_reg``/``end_reg`` f32, ``cls`` int64.

Batches that a dataset already produced in collated form (``CollatedBatch``, e.g. the dummy
dataset's vectorised ``__getitems__``) pass straight through.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch


class CollatedBatch(list):
    """[inputs, labels] (or [inputs, labels, items]) already in tensor form."""


def _token_types(tokens: np.ndarray, lengths: np.ndarray, sep_id: int, bert: bool) -> np.ndarray:
    B, L = tokens.shape
    if not bert:
        return np.zeros((B, L), dtype=np.int64)
    is_sep = tokens == sep_id
    first_sep = np.where(is_sep.any(1), is_sep.argmax(1), L)
    cols = np.arange(L)[None, :]
    return (cols > first_sep[:, None]).astype(np.int64)


def collate_fun(items: Sequence, tokenizer=None, return_items: bool = False, *, pad_token_id=None, sep_token_id=None,
                model_name=None):
    if isinstance(items, CollatedBatch):
        return items
    pad = pad_token_id if pad_token_id is not None else tokenizer.pad_token_id
    sep = sep_token_id if sep_token_id is not None else tokenizer.sep_token_id
    name = model_name if model_name is not None else getattr(tokenizer, "model_name", "bert")
    B = len(items)
    lengths = np.array([len(it.input_ids) for it in items], dtype=np.int64)
    L = int(lengths.max())
    tokens = np.full((B, L), pad, dtype=np.int64)
    for i, it in enumerate(items):
        tokens[i, :lengths[i]] = it.input_ids
    tt = _token_types(tokens, lengths, sep, name == "bert")
    inputs = {"input_ids": torch.from_numpy(tokens), "attention_mask": torch.from_numpy(tokens > 0),
              "token_type_ids": torch.from_numpy(tt)}
    labels = {"start_class": torch.tensor([it.start_id for it in items], dtype=torch.int64),
              "end_class": torch.tensor([it.end_id for it in items], dtype=torch.int64),
              "start_reg": torch.tensor([it.start_position for it in items], dtype=torch.float32),
              "end_reg": torch.tensor([it.end_position for it in items], dtype=torch.float32),
              "cls": torch.tensor([it.label_id for it in items], dtype=torch.int64)}
    if return_items:
        return [inputs, labels, list(items)]
    return [inputs, labels]


def merge_micro_batches(micro: Sequence, pad_token_id: int = 0):
    """One forward/backward batch from S collated micro-batches, keeping the reference's objective.

    Each micro-batch ``(inputs, labels)`` was collated on its own (padded to its own max length L_s, as
    ``collate_fun`` does per DataLoader batch).  They are right-padded to the longest L and concatenated; the
    extra positions are padding with ``attention_mask`` False (masked keys, so every real token's encoding is
    unchanged), and ``labels`` gains

    * ``segments`` — int32 [S] of the L_s, on the batch's device (read by the loss kernel, graph-capturable),
    * ``segment_lengths`` — the same as a tuple of ints (the CPU loss path),

    with which the loss scores segment s exactly as the reference scores micro-batch s (span softmax over its
    L_s positions, every term normalised inside the segment) and averages over segments (``models/losses.py
    WeightedLoss._segmented``; ``heads.hip`` ``qa_loss_kernel``).  All micro-batches must have the same size."""
    micro = list(micro)
    if len(micro) == 1:
        return micro[0]
    lens = [int(inp["input_ids"].shape[1]) for inp, _ in micro]
    sizes = {int(inp["input_ids"].shape[0]) for inp, _ in micro}
    assert len(sizes) == 1, f"micro-batches of unequal size {sorted(sizes)} cannot be merged into equal segments"
    Lm = max(lens)
    fill = {"input_ids": pad_token_id, "token_type_ids": 0, "attention_mask": False}

    def pad(t, key):
        if t.dim() < 2 or t.shape[1] == Lm:
            return t
        ext = torch.full((t.shape[0], Lm - t.shape[1]), fill.get(key, 0), dtype=t.dtype, device=t.device)
        return torch.cat([t, ext], 1)
    inputs = {k: torch.cat([pad(inp[k], k) for inp, _ in micro], 0) for k in micro[0][0]}
    labels = {k: torch.cat([lab[k] for _, lab in micro], 0) for k in micro[0][1]
              if torch.is_tensor(micro[0][1][k]) and k != "segments"}
    dev = inputs["input_ids"].device
    labels["segments"] = torch.tensor(lens, dtype=torch.int32).to(dev, non_blocking=True)
    labels["segment_lengths"] = tuple(lens)
    return inputs, labels
