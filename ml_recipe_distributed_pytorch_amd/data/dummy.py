"""Synthetic QA data (reference ``modules/model/dataset/dummy_dataset.py:6-51``).

Each item: ``[CLS] + q random ids + [SEP] + (L - q - 3) random ids + [SEP]`` (exactly
``max_seq_len`` tokens), ids uniform in ``[1, vocab)`` with pad/sep/cls remapped to unk, and
constant labels ``start_id=0, end_id=L-1, label_id=0 ('yes'), start_position=0, end_position=1``.

The reference builds items one by one in Python (0.34–0.47 ms/sample/core).  Here:
* ``DummyDataset.__getitems__`` (torch ≥ 2 batched fetch) synthesises a whole collated batch with
  vectorised numpy — the path the ``Trainer`` takes (CPU and GPU, through its DataLoader), and
* ``synth_batch_native`` uses the C++ generator in ``_hq_host`` (multi-threaded, writes straight
  into pinned tensors) — the path ``bench.py`` and ``smoke()`` use.
Both draw the same distribution; neither needs a vocab file (special ids come from the tokenizer
or the model preset).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from .collate import CollatedBatch, _token_types
from .items import DatasetItem


class SpecialIds:
    def __init__(self, vocab_size=30522, pad=0, unk=100, cls=101, sep=102, model_name="bert"):
        self.vocab_size, self.pad_token_id, self.unk_token_id = vocab_size, pad, unk
        self.cls_token_id, self.sep_token_id, self.model_name = cls, sep, model_name

    def __len__(self):
        return self.vocab_size

    @classmethod
    def from_tokenizer(cls, tok):
        return cls(len(tok), tok.pad_token_id, tok.unk_token_id, tok.cls_token_id, tok.sep_token_id,
                   getattr(tok, "model_name", "bert"))


def synth_ids(rng: np.random.Generator, B: int, L: int, q: int, sp: SpecialIds) -> np.ndarray:
    ids = rng.integers(1, sp.vocab_size, size=(B, L), dtype=np.int64)
    for w in (sp.pad_token_id, sp.sep_token_id, sp.cls_token_id):
        ids[ids == w] = sp.unk_token_id
    ids[:, 0] = sp.cls_token_id
    ids[:, q + 1] = sp.sep_token_id
    ids[:, L - 1] = sp.sep_token_id
    return ids


def make_batch(ids: np.ndarray, sp: SpecialIds, *, pin: bool = False):
    B, L = ids.shape
    tt = _token_types(ids, None, sp.sep_token_id, sp.model_name == "bert")
    t_ids = torch.from_numpy(ids)
    t_tt = torch.from_numpy(tt)
    mask = t_ids > 0
    labels = {"start_class": torch.zeros(B, dtype=torch.int64),
              "end_class": torch.full((B,), L - 1, dtype=torch.int64),
              "start_reg": torch.zeros(B, dtype=torch.float32),
              "end_reg": torch.ones(B, dtype=torch.float32),
              "cls": torch.zeros(B, dtype=torch.int64)}
    inputs = {"input_ids": t_ids, "attention_mask": mask, "token_type_ids": t_tt}
    if pin and torch.cuda.is_available():
        inputs = {k: v.pin_memory() for k, v in inputs.items()}
        labels = {k: v.pin_memory() for k, v in labels.items()}
    return CollatedBatch([inputs, labels])


def synth_batch_native(B: int, L: int, q: int, sp: SpecialIds, seed: int, *, pin: bool = True, threads: int = 4):
    """C++ generator (``_hq_host.synth_dummy``): fills pinned int64 ids / token types / bool mask."""
    from .._native import host
    pin = pin and torch.cuda.is_available()
    ids = torch.empty((B, L), dtype=torch.int64, pin_memory=pin)
    tt = torch.empty((B, L), dtype=torch.int64, pin_memory=pin)
    mask = torch.empty((B, L), dtype=torch.bool, pin_memory=pin)
    host().synth_dummy(ids.data_ptr(), tt.data_ptr(), mask.data_ptr(), B, L, q, sp.vocab_size, sp.pad_token_id,
                       sp.unk_token_id, sp.cls_token_id, sp.sep_token_id, sp.model_name == "bert", seed & 0xFFFFFFFFFFFF,
                       threads)
    labels = {"start_class": torch.zeros(B, dtype=torch.int64),
              "end_class": torch.full((B,), L - 1, dtype=torch.int64),
              "start_reg": torch.zeros(B, dtype=torch.float32),
              "end_reg": torch.ones(B, dtype=torch.float32),
              "cls": torch.zeros(B, dtype=torch.int64)}
    if pin:
        labels = {k: v.pin_memory() for k, v in labels.items()}
    return CollatedBatch([{"input_ids": ids, "attention_mask": mask, "token_type_ids": tt}, labels])


class DummyDataset:
    def __init__(self, tokenizer=None, *args, max_seq_len: int = 384, max_question_len: int = 64,
                 dataset_len: int = 10000, special_ids: Optional[SpecialIds] = None, seed: Optional[int] = None,
                 **kwargs):
        self.tokenizer = tokenizer
        self.dataset_len = dataset_len
        self.max_seq_len = max_seq_len
        self.max_question_len = max_question_len
        self.sp = special_ids or (SpecialIds.from_tokenizer(tokenizer) if tokenizer is not None else SpecialIds())
        self._rng = np.random.default_rng(seed)

    def __len__(self):
        return self.dataset_len

    def __getitem__(self, idx) -> DatasetItem:
        ids = synth_ids(np.random.default_rng(np.random.randint(0, 2 ** 31)), 1, self.max_seq_len,
                        self.max_question_len, self.sp)[0]
        return DatasetItem(example_id="None", input_ids=ids.tolist(), start_id=0, end_id=self.max_seq_len - 1,
                           label_id=0, start_position=0, end_position=1)

    def __getitems__(self, indices: Sequence[int]):
        seed = np.random.randint(0, 2 ** 31)
        ids = synth_ids(np.random.default_rng(seed), len(indices), self.max_seq_len, self.max_question_len, self.sp)
        return make_batch(ids, self.sp)


def _refill(batch, sp: SpecialIds, q: int, seed: int, threads: int = 4):
    """Regenerate the ids / token types / mask of a native batch in place (reuses its pinned buffers)."""
    from .._native import host
    inputs = batch[0]
    ids, tt, mask = inputs["input_ids"], inputs["token_type_ids"], inputs["attention_mask"]
    B, L = ids.shape
    host().synth_dummy(ids.data_ptr(), tt.data_ptr(), mask.data_ptr(), B, L, q, sp.vocab_size, sp.pad_token_id,
                       sp.unk_token_id, sp.cls_token_id, sp.sep_token_id, sp.model_name == "bert", seed & 0xFFFFFFFFFFFF,
                       threads)


class DummyChunkDataset:
    """Validation-side dummy data (``validate --dummy_dataset``, fix of D12): every "document" expands
    into ``n_chunks`` random windows shaped like ``ChunkDataset`` output (no NQ file or vocab needed)."""

    def __init__(self, tokenizer=None, *args, max_seq_len: int = 384, max_question_len: int = 64,
                 dataset_len: int = 1000, n_chunks: int = 3, special_ids: Optional[SpecialIds] = None, **kwargs):
        self.max_seq_len, self.max_question_len = max_seq_len, max_question_len
        self.dataset_len, self.n_chunks = dataset_len, n_chunks
        self.sp = special_ids or (SpecialIds.from_tokenizer(tokenizer) if tokenizer is not None else SpecialIds())

    def __len__(self):
        return self.dataset_len

    def __getitem__(self, idx):
        from .items import ChunkItem
        L, q = self.max_seq_len, self.max_question_len
        ids = synth_ids(np.random.default_rng(int(idx)), self.n_chunks, L, q, self.sp)
        doc_len = L - q - 3
        items = []
        for c in range(self.n_chunks):
            items.append(ChunkItem(item_id=f"dummy-{idx}", input_ids=ids[c].tolist(), start_id=q + 2, end_id=L - 2,
                                   label_id=0, true_text="", true_question="", true_label=0, true_start=c * doc_len,
                                   true_end=c * doc_len + doc_len - 1, question_len=q, t2o=[],
                                   chunk_start=c * doc_len, chunk_end=(c + 1) * doc_len,
                                   start_position=(q + 2) / L, end_position=(L - 2) / L))
        return items
