"""Dataset item records and the label vocabulary (reference ``split_dataset.py:50-52,191-199`` and
``validation_dataset.py:15-39``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

LABELS = ["yes", "no", "short", "long", "unknown"]
LABELS2ID = {k: i for i, k in enumerate(LABELS)}
ID2LABELS = {i: k for k, i in LABELS2ID.items()}


@dataclass
class DatasetItem:
    example_id: str
    input_ids: List[int]
    start_id: int
    end_id: int
    label_id: int
    start_position: float
    end_position: float


@dataclass
class ChunkItem:
    item_id: str
    input_ids: List[int]
    start_id: int
    end_id: int
    label_id: int
    true_text: str
    true_question: str
    true_label: int
    true_start: int
    true_end: int
    question_len: int
    t2o: List[int] = field(default_factory=list)
    chunk_start: int = 0
    chunk_end: int = 0
    start_position: float = 0.0
    end_position: float = 0.0
