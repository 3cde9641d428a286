"""Data layer: dummy data (Python + native), collate, NQ preprocessing / windows, sentence splitter,
list loader (error propagation, D19), predictor scoring."""
import os

import numpy as np
import pytest
import torch

from conftest import FIXTURES
from ml_recipe_distributed_pytorch_amd.data.collate import collate_fun
from ml_recipe_distributed_pytorch_amd.data.dummy import (DummyChunkDataset, DummyDataset, SpecialIds, _refill,
                                                          synth_batch_native)
from ml_recipe_distributed_pytorch_amd.data.items import LABELS2ID, DatasetItem
from ml_recipe_distributed_pytorch_amd.data.list_loader import ListDataloader
from ml_recipe_distributed_pytorch_amd.data.sentences import split_sentences


# ------------------------------------------------------------------------------------------ dummy
def _check_dummy_batch(inputs, labels, L, q, sp):
    ids = inputs["input_ids"]
    assert ids.shape[1] == L and ids.dtype == torch.int64
    assert (ids[:, 0] == sp.cls_token_id).all() and (ids[:, q + 1] == sp.sep_token_id).all()
    assert (ids[:, L - 1] == sp.sep_token_id).all()
    body = torch.cat([ids[:, 1:q + 1], ids[:, q + 2:L - 1]], 1)
    for special in (sp.pad_token_id, sp.cls_token_id, sp.sep_token_id):
        assert not (body == special).any()
    assert (body >= 1).all() and (body < sp.vocab_size).all()
    tt = inputs["token_type_ids"]
    assert (tt[:, :q + 2] == 0).all() and (tt[:, q + 2:] == 1).all()
    assert inputs["attention_mask"].all()
    assert (labels["start_class"] == 0).all() and (labels["end_class"] == L - 1).all()
    assert (labels["cls"] == 0).all() and (labels["start_reg"] == 0).all() and (labels["end_reg"] == 1).all()


def test_dummy_dataset_item_and_batch():
    sp = SpecialIds()
    ds = DummyDataset(max_seq_len=64, max_question_len=16, dataset_len=10)
    it = ds[0]
    assert isinstance(it, DatasetItem) and len(it.input_ids) == 64 and it.end_id == 63 and it.label_id == 0
    b = collate_fun([ds[i] for i in range(4)], pad_token_id=0, sep_token_id=102, model_name="bert")
    _check_dummy_batch(b[0], b[1], 64, 16, sp)
    inputs, labels = ds.__getitems__(list(range(8)))
    _check_dummy_batch(inputs, labels, 64, 16, sp)


def test_native_dummy_batch(host_lib):
    sp = SpecialIds()
    b = synth_batch_native(16, 128, 64, sp, seed=3, pin=False)
    _check_dummy_batch(b[0], b[1], 128, 64, sp)
    before = b[0]["input_ids"].clone()
    _refill(b, sp, 64, seed=4)
    assert not torch.equal(before, b[0]["input_ids"])
    _check_dummy_batch(b[0], b[1], 128, 64, sp)
    again = synth_batch_native(16, 128, 64, sp, seed=3, pin=False)
    assert torch.equal(before, again[0]["input_ids"])  # deterministic per seed
    ids = synth_batch_native(64, 384, 64, sp, seed=5, pin=False)[0]["input_ids"][:, 1:65].flatten().float()
    # roughly uniform over the vocab
    assert abs(ids.mean().item() / (sp.vocab_size / 2) - 1) < 0.02


def test_collate_padding_and_token_types():
    items = [DatasetItem("a", [101, 5, 6, 102, 7, 8, 102], 4, 5, 2, 0.1, 0.2),
             DatasetItem("b", [101, 9, 102, 10, 102], -1, -1, 4, -0.1, -0.1)]
    inputs, labels = collate_fun(items, pad_token_id=0, sep_token_id=102, model_name="bert")
    assert inputs["input_ids"].tolist() == [[101, 5, 6, 102, 7, 8, 102], [101, 9, 102, 10, 102, 0, 0]]
    assert inputs["token_type_ids"].tolist() == [[0, 0, 0, 0, 1, 1, 1], [0, 0, 0, 1, 1, 1, 1]]
    assert inputs["attention_mask"].tolist()[1] == [True] * 5 + [False] * 2
    assert labels["start_class"].tolist() == [4, -1] and labels["cls"].tolist() == [2, 4]
    r_inputs, _ = collate_fun(items, pad_token_id=1, sep_token_id=2, model_name="roberta")
    assert (r_inputs["token_type_ids"] == 0).all()


def test_dummy_chunk_dataset():
    ds = DummyChunkDataset(max_seq_len=32, max_question_len=8, dataset_len=3, n_chunks=2)
    chunks = ds[1]
    assert len(chunks) == 2 and all(len(c.input_ids) == 32 for c in chunks)
    assert chunks[0].item_id == chunks[1].item_id and chunks[0].question_len == 8


# ------------------------------------------------------------------------------------ sentences
def test_split_sentences():
    t = "Dr. Smith went to Washington. He arrived at 5 p.m. on Monday! Did he stay? Yes. <P> Next para."
    s = split_sentences(t)
    assert s[0] == "Dr. Smith went to Washington."
    assert "".join(x.replace(" ", "") for x in s) == t.replace(" ", "")
    assert any(x.startswith("Did he stay?") for x in s)
    assert split_sentences("") == [""]
    assert split_sentences("no terminal punctuation") == ["no terminal punctuation"]


# ------------------------------------------------------------------------------------------- NQ
@pytest.fixture(scope="module")
def nq(tmp_path_factory, host_lib):
    from ml_recipe_distributed_pytorch_amd.data.nq import RawPreprocessor
    from ml_recipe_distributed_pytorch_amd.data.synth_nq import write_jsonl
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    d = tmp_path_factory.mktemp("nq")
    vocab = os.path.join(FIXTURES, "toy_vocab.txt")
    write_jsonl(str(d / "nq.jsonl"), 60, seed=1, vocab_file=vocab)
    pre = RawPreprocessor(str(d / "nq.jsonl"), str(d / "proc"))
    out = pre()
    tok = Tokenizer("bert", vocab)
    return d, out, tok


def test_preprocessor_labels_and_split(nq):
    from ml_recipe_distributed_pytorch_amd.data.nq import RawPreprocessor
    d, (counter, labels, (tr, trl, te, tel)), _ = nq
    assert len(labels) == 60 and sum(counter.values()) == 60
    assert sorted(np.concatenate([tr, te]).tolist()) == list(range(60))
    assert (labels[tr] == trl).all() and (labels[te] == tel).all()
    for y, n in counter.items():  # stratified: every class with ≥ 2 docs keeps train members
        assert (trl == y).sum() >= n - max(1, int(np.ceil(0.05 * n)))
    # second call loads the JSON caches and returns identical results
    c2, l2, (tr2, _, te2, _) = RawPreprocessor(str(d / "nq.jsonl"), str(d / "proc"))()
    assert c2 == counter and (l2 == labels).all() and (tr2 == tr).all() and (te2 == te).all()
    assert (d / "proc" / "label.info").exists() and (d / "proc" / "split.info").exists()


def test_reference_prepared_directory_is_reused_without_unpickling(nq, tmp_path):
    """A processed_data_path written by the reference: {i}.json examples (same format) + PICKLED
    label.info / split.info.  The pickles are detected by their first byte and never loaded; labels come
    from the example files, the split is recomputed (same per-class random_state=0 rule), JSON side files
    hold the caches, and the reference's files are left byte-identical."""
    import pickle
    import shutil
    from ml_recipe_distributed_pytorch_amd.data.nq import RawPreprocessor
    d, (counter, labels, (tr, trl, te, tel)), _ = nq
    ref_dir = tmp_path / "ref_proc"
    ref_dir.mkdir()
    for i in range(len(labels)):
        shutil.copy(d / "proc" / f"{i}.json", ref_dir / f"{i}.json")
    blobs = {"label.info": pickle.dumps(({0: 1}, np.zeros(3)), protocol=4),   # content deliberately wrong:
             "split.info": pickle.dumps((np.zeros(1),) * 4, protocol=4)}       # it must never be read
    for name, b in blobs.items():
        (ref_dir / name).write_bytes(b)
    pre = RawPreprocessor(str(d / "missing.jsonl"), str(ref_dir))   # no raw pass: the jsonl is not needed
    assert pre.from_reference
    c2, l2, (tr2, trl2, te2, tel2) = pre()
    assert c2 == counter and (l2 == labels).all()
    assert (tr2 == tr).all() and (te2 == te).all() and (trl2 == trl).all() and (tel2 == tel).all()
    for name, b in blobs.items():
        assert (ref_dir / name).read_bytes() == b
        assert (ref_dir / (name + ".json")).exists()
    c3, l3, _ = RawPreprocessor(str(d / "missing.jsonl"), str(ref_dir))()   # second run: the side files
    assert c3 == counter and (l3 == labels).all()


def _answer_text(tok, line):
    from ml_recipe_distributed_pytorch_amd.data.nq import RawPreprocessor
    _, s, e = RawPreprocessor._get_target(line)
    words = [w for w in line["document_text"].split()[s:e] if not (w.startswith("<") and w.endswith(">"))]
    return tok.decode([t for w in words for t in tok.encode(w)])


@pytest.mark.parametrize("by_sentence", [False, True])
def test_split_dataset_windows(nq, by_sentence):
    from ml_recipe_distributed_pytorch_amd.data.nq import SplitDataset
    d, (_, _, (tr, *_)), tok = nq
    L = 96
    ds = SplitDataset(str(d / "proc"), tok, tr, max_seq_len=L, max_question_len=16, doc_stride=24,
                      split_by_sentence=by_sentence, truncate=True, test=True)
    n_span = 0
    for i in range(len(ds)):
        it = ds[i]
        assert len(it.input_ids) <= L
        assert it.input_ids[0] == tok.cls_token_id and it.input_ids[-1] == tok.sep_token_id
        if it.start_id >= 0:
            assert it.label_id != LABELS2ID["unknown"]
            got = tok.decode(it.input_ids[it.start_id:it.end_id])
            exp = _answer_text(tok, ds._load(i))
            if it.end_id < len(it.input_ids) - 1:
                assert got == exp
            n_span += 1
        else:
            assert it.label_id == LABELS2ID["unknown"]
    assert n_span > 0


def test_split_dataset_sampling_prefers_answers(nq):
    from ml_recipe_distributed_pytorch_amd.data.nq import SplitDataset
    d, (_, labels, (tr, *_)), tok = nq
    ds = SplitDataset(str(d / "proc"), tok, tr, max_seq_len=64, max_question_len=16, doc_stride=16)
    np.random.seed(0)
    short = [i for i, j in enumerate(tr) if labels[j] == LABELS2ID["short"]]
    hits = sum(ds[i].start_id >= 0 for i in short)
    assert hits == len(short)  # a window containing the short answer always exists and dominates (1 vs 1e-3)


def test_chunk_dataset_covers_document(nq):
    from ml_recipe_distributed_pytorch_amd.data.nq import ChunkDataset, encode_document
    d, (_, _, (_, _, te, _)), tok = nq
    ds = ChunkDataset(str(d / "proc"), tok, te, max_seq_len=64, max_question_len=16, doc_stride=16)
    for i in range(len(ds)):
        chunks = ds[i]
        line = ds._load(i)
        doc = encode_document(tok, line["document_text"])
        assert chunks[0].chunk_start == 0
        assert chunks[-1].chunk_end >= len(doc.tokens)
        assert all(c.item_id == line["example_id"] for c in chunks)
        assert all(c.t2o == doc.t2o for c in chunks)


# ---------------------------------------------------------------------------------- list loader
class _Docs:
    def __init__(self, n, bad=None):
        self.n, self.bad = n, bad

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if i == self.bad:
            raise ValueError(f"broken document {i}")
        return [(i, k) for k in range(i % 3 + 1)]


@pytest.mark.parametrize("n_jobs", [0, 2])
def test_list_loader_yields_every_chunk(n_jobs):
    dl = ListDataloader(_Docs(20), batch_size=4, n_jobs=n_jobs, shuffle=True, seed=0)
    got = [c for b in dl for c in b]
    assert sorted(got) == sorted((i, k) for i in range(20) for k in range(i % 3 + 1))
    assert all(len(b) == 4 for b in list(dl)[:-1])


def test_list_loader_propagates_worker_errors():
    dl = ListDataloader(_Docs(20, bad=7), batch_size=4, n_jobs=2, timeout_s=60)
    with pytest.raises(ValueError, match="broken document 7"):
        list(dl)


# ------------------------------------------------------------------------------------ predictor
def test_predictor_candidate_rules():
    from ml_recipe_distributed_pytorch_amd.data.items import ChunkItem
    from ml_recipe_distributed_pytorch_amd.infer.predictor import Predictor

    class _M(torch.nn.Module):
        def forward(self, **kw):
            raise AssertionError

    p = Predictor(_M(), "cpu", n_jobs=0)
    mk = lambda cs: ChunkItem("d", [0] * 10, 0, 0, 0, "a b c d e f", "q", 2, 3, 5, question_len=2, t2o=list(range(6)),
                              chunk_start=cs)
    a, b = mk(0), mk(0)
    # start before the document part (q_len + 2 = 4) is invalid; start > end invalid
    p._update_candidates([5.0, 6.0, 1.0], [3, 7, 5], [6, 6, 7], [0.1] * 3, [0.2] * 3, [2, 2, 3], [a, b, a])
    assert "d" in p.candidates and p.candidates["d"].start_id == 5 and p.scores["d"] == 1.0
    p._update_candidates([4.0], [6], [8], [0.0], [0.0], [2], [b])
    assert p.candidates["d"].start_id == 6
    p._update_candidates([0.5], [4], [5], [0.0], [0.0], [1], [b])  # lower score loses
    assert p.candidates["d"].start_id == 6
    m = p.metrics()
    assert m["documents"] == 1 and m["label_accuracy"] == 1.0
    assert p.predicted_text("d") == "c d e"
