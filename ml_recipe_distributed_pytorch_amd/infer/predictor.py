"""Chunked QA inference (reference ``modules/model/inference/predictor.py:14-144``).

For every chunk of every document: argmax start / end logits, softmax-argmax class, and the
score of arXiv:1901.08634 ``max_start + max_end − (start[CLS] + end[CLS])``.  Per document the best
*valid* chunk wins (start ≤ end, start inside the document part ``≥ question_len + 2``, score not
below the best so far).  Scoring is vectorised per batch on device; a single device→host copy per
batch carries everything the candidate update needs.

Additions (D12): ``metrics()`` — label accuracy, span exact-match / token-F1 against the true
document-token span, and coverage — and ``predicted_text`` for ``show_predictions``.
"""
from __future__ import annotations

import json
import logging
from collections import defaultdict
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from ..data.items import ID2LABELS
from ..data.list_loader import ListDataloader
from ..train.engine import to_device

logger = logging.getLogger(__name__)


@dataclass
class PredictorCandidate:
    start_id: int
    end_id: int
    start_reg: float
    end_reg: float
    label: int
    score: float = 0.0


def doc_span(item, start_id: int, end_id: int):
    """Chunk token positions → document token positions."""
    off = item.chunk_start - (item.question_len + 2)
    return start_id + off, end_id + off


class Predictor:
    def __init__(self, model, device, *, batch_size=256, n_jobs=16, collate_fun=None, buffer_size=4096, limit=None,
                 timeout_s: float = 600.0):
        self.model = model
        self.device = torch.device(device)
        self.model.to(self.device)
        self.scores: Dict[str, float] = defaultdict(float)
        self.candidates: Dict[str, PredictorCandidate] = {}
        self.items = {}
        self.batch_size, self.n_jobs, self.collate_fun = batch_size, n_jobs, collate_fun
        self.buffer_size, self.limit, self.timeout_s = buffer_size, limit, timeout_s
        self.dump = None
        self.n_chunks = 0
        logger.info(f"Predictor uses {self.device} device. Batch size: {self.batch_size}. #workers: {self.n_jobs}. "
                    f"Buffer size: {self.buffer_size}. Set limit: {self.limit}.")

    def _is_valid(self, item, score, start_id, end_id) -> bool:
        assert score >= 0
        if start_id > end_id or start_id < item.question_len + 2:
            return False
        return not (self.scores[item.item_id] > score)

    def _update_candidates(self, scores, start_ids, end_ids, start_regs, end_regs, labels, items):
        for sc, s, e, sr, er, lb, item in zip(scores, start_ids, end_ids, start_regs, end_regs, labels, items):
            if self._is_valid(item, sc, s, e):
                self.scores[item.item_id] = float(sc)
                self.candidates[item.item_id] = PredictorCandidate(int(s), int(e), float(sr), float(er), int(lb),
                                                                   float(sc))
                self.items[item.item_id] = item

    @staticmethod
    def score_batch(preds):
        """Device-side scoring → one [B, 6] float64 host array (score, start, end, sreg, ereg, cls)."""
        sp, ep = preds["start_class"].float(), preds["end_class"].float()
        s_logit, s_id = sp.max(-1)
        e_logit, e_id = ep.max(-1)
        cls_id = torch.softmax(preds["cls"].float(), -1).argmax(-1)
        score = s_logit + e_logit - (sp[:, 0] + ep[:, 0])
        out = torch.stack([score, s_id.float(), e_id.float(), preds["start_reg"].float().reshape(-1),
                           preds["end_reg"].float().reshape(-1), cls_id.float()], 1)
        return out.double().cpu().numpy()

    @torch.no_grad()
    def __call__(self, dataset, *, save_dump=False):
        self.model.eval()
        loader = ListDataloader(dataset, batch_size=self.batch_size, n_jobs=self.n_jobs, collate_fun=self.collate_fun,
                                buffer_size=self.buffer_size, shuffle=True, timeout_s=self.timeout_s)
        if save_dump:
            self.dump = []
        for batch_i, (inputs, _labels, items) in enumerate(loader):
            inputs = to_device(inputs, self.device)
            r = self.score_batch(self.model(**inputs))
            self.n_chunks += len(items)
            self._update_candidates(r[:, 0], r[:, 1].astype(np.int64), r[:, 2].astype(np.int64), r[:, 3], r[:, 4],
                                    r[:, 5].astype(np.int64), items)
            if save_dump:
                self.dump.append((r[:, 0], r[:, 1].astype(np.int64), r[:, 2].astype(np.int64),
                                  r[:, 5].astype(np.int64), [it.item_id for it in items]))
            if self.limit is not None and batch_i >= self.limit:
                break
        return self

    # ------------------------------------------------------------------------------------ reporting
    def predicted_text(self, item_id) -> str:
        item, c = self.items[item_id], self.candidates[item_id]
        ds, de = doc_span(item, c.start_id, c.end_id)
        if not item.t2o:
            return ""
        words = item.true_text.split()
        w0 = item.t2o[min(max(ds, 0), len(item.t2o) - 1)]
        w1 = item.t2o[min(max(de, 0), len(item.t2o) - 1)]
        return " ".join(words[w0:w1 + 1])

    def metrics(self) -> Dict[str, float]:
        n = len(self.candidates)
        if n == 0:
            return {"documents": 0, "chunks": self.n_chunks}
        acc = em = f1 = 0.0
        n_span = 0
        for k, c in self.candidates.items():
            item = self.items[k]
            acc += float(c.label == item.true_label)
            if item.true_start >= 0:
                n_span += 1
                ps, pe = doc_span(item, c.start_id, c.end_id)
                ts, te = item.true_start, item.true_end
                em += float(ps == ts and pe == te)
                inter = max(0, min(pe, te) - max(ps, ts))
                if inter > 0:
                    p, r = inter / max(pe - ps, 1), inter / max(te - ts, 1)
                    f1 += 2 * p * r / (p + r)
        return {"documents": n, "chunks": self.n_chunks, "label_accuracy": acc / n,
                "span_exact": em / max(n_span, 1), "span_f1": f1 / max(n_span, 1), "span_documents": n_span}

    def show_predictions(self, *, n_docs=None):
        for doc_i, doc_id in enumerate(self.scores.keys()):
            if n_docs is not None and doc_i >= n_docs:
                break
            doc, cand = self.items[doc_id], self.candidates[doc_id]
            logger.info(f"Text: {doc.true_text}")
            logger.info(f"Question: {doc.true_question}")
            logger.info(f"True label: {ID2LABELS[doc.true_label]}. Pred label: {ID2LABELS[cand.label]}.")
            logger.info(f"Predicted answer: {self.predicted_text(doc_id)}")

    def save_predictions(self, path: str):
        out = {str(k): {"label": ID2LABELS[c.label], "score": c.score, "start_id": c.start_id, "end_id": c.end_id,
                        "start_reg": c.start_reg, "end_reg": c.end_reg, "text": self.predicted_text(k)}
               for k, c in self.candidates.items()}
        with open(path, "w") as f:
            json.dump({"metrics": self.metrics(), "predictions": out}, f, indent=1)
