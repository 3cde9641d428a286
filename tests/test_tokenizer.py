"""Native C++ WordPiece / byte-level BPE vs the HF ``tokenizers`` library on the same vocab files."""
import os

import pytest

from conftest import FIXTURES

tokenizers = pytest.importorskip("tokenizers")

TEXTS = [
    "The quick brown fox jumps over the lazy dog!",
    "Hello, World. naïve café résumé — unbelievable",
    "New York City is big; when was it built? 1231 a-b (c)",
    "中国人 hello\tworld\n  spaces   ",
    "<P> tags </P> and ##hash x1 x2 unknownwordzz",
    "",
    "ÀÉÎõü ǅ ﬁ Ⅻ ① ½",
]


@pytest.fixture(scope="module")
def wp(host_lib):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    return Tokenizer("bert", os.path.join(FIXTURES, "toy_vocab.txt"), lowercase=True)


@pytest.mark.parametrize("lower,chinese", [(True, False), (False, True), (True, True)])
def test_wordpiece_matches_hf(host_lib, lower, chinese):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    vocab = os.path.join(FIXTURES, "toy_vocab.txt")
    ours = Tokenizer("bert", vocab, lowercase=lower, handle_chinese_chars=chinese)
    ref = tokenizers.BertWordPieceTokenizer(vocab, lowercase=lower, handle_chinese_chars=chinese)
    for t in TEXTS:
        exp = ref.encode(t, add_special_tokens=False).ids
        assert ours.encode(t) == exp, t
    assert ours.encode_batch(TEXTS) == [ref.encode(t, add_special_tokens=False).ids for t in TEXTS]


def test_wordpiece_legacy_mode_wraps_specials(host_lib):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    vocab = os.path.join(FIXTURES, "toy_vocab.txt")
    ours = Tokenizer("bert", vocab, legacy=True)
    ref = tokenizers.BertWordPieceTokenizer(vocab, lowercase=True)
    assert ours.encode("hello world") == ref.encode("hello world").ids  # [CLS] … [SEP] (reference D11)


def test_special_ids_and_decode(wp):
    assert (wp.pad_token_id, wp.unk_token_id, wp.cls_token_id, wp.sep_token_id) == (0, 1, 2, 3)
    ids = wp.encode("the quick fox jumps")
    assert wp.decode([wp.cls_token_id] + ids + [wp.sep_token_id]) == "the quick fox jumps"


def test_pickle_roundtrip(wp):
    import pickle
    clone = pickle.loads(pickle.dumps(wp))
    assert clone.encode_batch(TEXTS) == wp.encode_batch(TEXTS)


def test_bpe_matches_hf(host_lib):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    v = os.path.join(FIXTURES, "toy_bpe", "vocab.json")
    m = os.path.join(FIXTURES, "toy_bpe", "merges.txt")
    ours = Tokenizer("roberta", v, merges_file=m)
    ref = tokenizers.ByteLevelBPETokenizer(v, m)
    for t in TEXTS + ["  leading spaces", "it's they're we'll I'm", "tabs\tand\nnewlines"]:
        assert ours.encode(t) == ref.encode(t).ids, t
        assert ours.decode(ours.encode(t)) == ref.decode(ref.encode(t).ids), t


def test_bpe_requires_merges(host_lib):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    with pytest.raises(AttributeError):
        Tokenizer("roberta", os.path.join(FIXTURES, "toy_bpe", "vocab.json"))


def test_bpe_dropout_changes_segmentation_but_not_text(host_lib):
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    v = os.path.join(FIXTURES, "toy_bpe", "vocab.json")
    m = os.path.join(FIXTURES, "toy_bpe", "merges.txt")
    full = Tokenizer("roberta", v, merges_file=m)
    drop = Tokenizer("roberta", v, merges_file=m, dropout=0.5, seed=1)
    t = "The quick brown fox jumps over the lazy dog " * 4
    outs = {tuple(drop.encode(t)) for _ in range(8)}
    assert len(outs) > 1
    for o in outs:
        assert drop.decode(list(o)) == full.decode(full.encode(t))
        assert len(o) >= len(full.encode(t))
