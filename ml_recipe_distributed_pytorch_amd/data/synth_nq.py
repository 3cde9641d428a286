"""Synthetic Natural-Questions jsonl generator (same schema as the Kaggle ``simplified-nq-train.jsonl``
the reference trains on; there is no network to fetch the real file).

Documents are HTML-tagged paragraphs (``<P> … </P>``, ``<Table>``…) of words drawn from a vocabulary
file (or a built-in word list), with a question, long-answer candidates = the paragraphs, and one
annotation whose type is drawn from yes/no/short/long/unknown.  Used by the CPU tests, the CLI
smoke runs and ``validate`` demos.

    python -m ml_recipe_distributed_pytorch_amd.data.synth_nq out.jsonl --n 200 [--vocab vocab.txt]
"""
from __future__ import annotations

import argparse
import json
from typing import List, Optional

import numpy as np

_WORDS = ("the of and to in is was for on as with by at from his an were are which this be has had it "
          "one new first city year time world state people war team game film series season river music "
          "school house party album song station university company church county national north south "
          "history number water village family government system during after before between under").split()


def _vocab_words(vocab_file: Optional[str]) -> List[str]:
    if not vocab_file:
        return list(_WORDS)
    words = []
    with open(vocab_file, encoding="utf-8") as f:
        for line in f:
            w = line.rstrip("\n")
            if w.isalpha() and w.islower() and len(w) > 1:
                words.append(w)
    return words or list(_WORDS)


# learnable mode: the question names a KEY word that appears exactly once in the document — at the short answer's
# start / as the answer paragraph's first word — and a CLASS word that gives the annotation type, so span and
# class can only be predicted by matching question to document (a task random-init BERT can learn in a few
# hundred steps; used by tools/fp8_convergence.py for the fp8-vs-bf16 comparison)
KEY_WORDS = [f"key{i}" for i in range(64)]
CLASS_WORDS = ["yesq", "noq", "shortq", "longq", "noneq"]


def learnable_vocab(path: str) -> str:
    """A WordPiece vocab covering the built-in words, the key words and the class words."""
    with open(path, "w") as f:
        for w in ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "."] + list(_WORDS) + KEY_WORDS + CLASS_WORDS:
            f.write(w + "\n")
    return path


def make_example(rng: np.random.Generator, words: List[str], idx: int, *, n_par=(2, 8), par_len=(8, 60),
                 label_p=(0.05, 0.05, 0.3, 0.3, 0.3), learnable: bool = False) -> dict:
    if learnable:
        return _make_learnable(rng, words, idx, n_par=n_par, par_len=par_len, label_p=label_p)
    toks, cands = [], []
    for _ in range(int(rng.integers(*n_par))):
        tag = "P" if rng.random() < 0.85 else "Table"
        start = len(toks)
        toks.append(f"<{tag}>")
        n = int(rng.integers(*par_len))
        for j in range(n):
            w = words[int(rng.integers(len(words)))]
            if j == 0 or (j > 3 and rng.random() < 0.08):
                w = w.capitalize()
            if rng.random() < 0.08 and j < n - 1:
                w += "."
            toks.append(w)
        toks[-1] += "."
        toks.append(f"</{tag}>")
        cands.append({"start_token": start, "end_token": len(toks), "top_level": True})
    question = " ".join(words[int(rng.integers(len(words)))] for _ in range(int(rng.integers(4, 12))))
    kind = ["yes", "no", "short", "long", "unknown"][int(rng.choice(5, p=np.asarray(label_p) / sum(label_p)))]
    ann = {"yes_no_answer": "NONE", "long_answer": {"start_token": -1, "end_token": -1, "candidate_index": -1},
           "short_answers": [], "annotation_id": int(rng.integers(1 << 62))}
    if kind != "unknown":
        ci = int(rng.integers(len(cands)))
        c = cands[ci]
        ann["long_answer"] = {"start_token": c["start_token"], "end_token": c["end_token"], "candidate_index": ci}
        if kind in ("yes", "no"):
            ann["yes_no_answer"] = kind.upper()
        elif kind == "short":
            s = int(rng.integers(c["start_token"] + 1, c["end_token"] - 1))
            e = min(s + int(rng.integers(1, 5)), c["end_token"] - 1)
            ann["short_answers"] = [{"start_token": s, "end_token": e}]
    return {"document_text": " ".join(toks), "long_answer_candidates": cands, "question_text": question,
            "annotations": [ann], "document_url": f"https://example.invalid/{idx}",
            "example_id": int(5_000_000_000_000_000_000 + idx)}


def _make_learnable(rng, words, idx, *, n_par, par_len, label_p) -> dict:
    kind_i = int(rng.choice(5, p=np.asarray(label_p) / sum(label_p)))
    kind = ["yes", "no", "short", "long", "unknown"][kind_i]
    key = KEY_WORDS[int(rng.integers(len(KEY_WORDS)))]
    pars = []
    for _ in range(int(rng.integers(*n_par))):
        pars.append([words[int(rng.integers(len(words)))] for _ in range(int(rng.integers(*par_len)))])
    ci = int(rng.integers(len(pars)))
    short = None
    if kind != "unknown":
        p = pars[ci]
        pos = 0 if kind in ("long", "yes", "no") else int(rng.integers(0, max(1, len(p) - 4)))
        p[pos] = key
        short = (pos, min(pos + int(rng.integers(1, 4)), len(p)))
    toks, cands = [], []
    for i, p in enumerate(pars):
        start = len(toks)
        toks.append("<P>")
        if i == ci and short is not None:
            s_tok = len(toks) + short[0]
            e_tok = len(toks) + short[1]
        toks.extend(p)
        toks.append("</P>")
        cands.append({"start_token": start, "end_token": len(toks), "top_level": True})
    q = [words[int(rng.integers(len(words)))] for _ in range(int(rng.integers(3, 8)))]
    q.insert(int(rng.integers(len(q) + 1)), key)
    q.insert(int(rng.integers(len(q) + 1)), CLASS_WORDS[kind_i])
    ann = {"yes_no_answer": "NONE", "long_answer": {"start_token": -1, "end_token": -1, "candidate_index": -1},
           "short_answers": [], "annotation_id": int(rng.integers(1 << 62))}
    if kind != "unknown":
        c = cands[ci]
        ann["long_answer"] = {"start_token": c["start_token"], "end_token": c["end_token"], "candidate_index": ci}
        if kind in ("yes", "no"):
            ann["yes_no_answer"] = kind.upper()
        elif kind == "short":
            ann["short_answers"] = [{"start_token": s_tok, "end_token": e_tok}]
    return {"document_text": " ".join(toks), "long_answer_candidates": cands, "question_text": " ".join(q),
            "annotations": [ann], "document_url": f"https://example.invalid/{idx}",
            "example_id": int(5_000_000_000_000_000_000 + idx)}


def write_jsonl(path: str, n: int, *, seed: int = 0, vocab_file: Optional[str] = None, **kw) -> str:
    rng = np.random.default_rng(seed)
    words = _vocab_words(vocab_file)
    with open(path, "w") as f:
        for i in range(n):
            f.write(json.dumps(make_example(rng, words, i, **kw)) + "\n")
    return path


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--vocab", default=None)
    a = ap.parse_args(argv)
    write_jsonl(a.out, a.n, seed=a.seed, vocab_file=a.vocab)


if __name__ == "__main__":
    main()
