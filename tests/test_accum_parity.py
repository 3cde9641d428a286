"""Gradient accumulation semantics (reference ``trainer.py:197-204,284``): one optimizer step over
``batch_split`` micro-batches accumulates ∇(loss(micro) / batch_split) — the mean of per-micro-batch means.
With ignored spans (start/end class −1: CE averages over the VALID spans of each micro-batch) that is not the
gradient of a plainly merged batch ('merge'), but it IS the gradient of the segmented merge
(``merge_micro_batches`` + the loss's segment mode), which the GPU default uses: the micro-batches keep their
own padded lengths, valid-span counts and class normalisers as loss segments."""
import pytest
import torch

from test_dist_cpu import _batch, _build, _split


def _with_ignored_spans(batch):
    inputs, labels = batch
    labels = dict(labels)
    sc, ec = labels["start_class"].clone(), labels["end_class"].clone()
    sc[[1, 2, 3]] = -1   # first half: 1 valid span of 4, second half: 4 of 4
    ec[[1, 2, 3]] = -1
    labels["start_class"], labels["end_class"] = sc, ec
    return inputs, labels


def _grads(model, loss_fn, batch, split):
    model.zero_grad()
    for i in range(split):
        inp, lab = _split(batch, split, i)
        (loss_fn(model(**inp), lab) / split).backward()
    return model.store.grad.clone()


def test_engine_accumulation_is_mean_of_micro_batch_means():
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    torch.manual_seed(0)
    model, loss_fn, opt = _build(3)
    batch = _with_ignored_spans(_batch(B=8, L=32, seed=4))
    ref = _grads(model, loss_fn, batch, 2)
    merged = _grads(model, loss_fn, batch, 1)
    # the two objectives really differ on this batch (that difference is what 'merge' changes)
    assert (ref - merged).norm() / ref.norm() > 1e-2
    eng = TrainEngine(model, loss_fn, opt, batch_split=2, max_grad_norm=0.0)
    seen = {}
    orig = opt.step

    def spy(**kw):
        seen["g"] = model.store.grad.clone()
        return orig(**kw)
    opt.step = spy
    model.zero_grad()   # the manual backward passes above left the arena "accumulating"
    eng.step([_split(batch, 2, 0), _split(batch, 2, 1)])
    torch.testing.assert_close(seen["g"], ref, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("val,expect", [(None, None), ("True", True), ("merge", "merge"), ("raise", "raise"),
                                        ("False", False)])
def test_auto_batch_split_values(val, expect):
    from ml_recipe_distributed_pytorch_amd.utils.flags import get_trainer_parser
    argv = ["--data_path", "x", "--processed_data_path", "y", "--experiment_name", "e"]
    if val is not None:
        argv += ["--auto_batch_split", val]
    ns, _ = get_trainer_parser().parse_known_args(argv)
    assert ns.auto_batch_split == expect


def test_plan_never_lowers_the_split_unless_merging():
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.train.memory import plan_batch_split
    cfg = get_config("bert-base-uncased")
    assert plan_batch_split(cfg, 512, 256, 288 * 2**30, requested=128, merge=False) == 128
    assert plan_batch_split(cfg, 512, 256, 288 * 2**30, requested=128, merge=True) == 1


def _loss(kind, label_weights=False):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    lp = SimpleNamespace(loss=kind, smooth_alpha=0.1, focal_alpha=1.0, focal_gamma=2.0, w_start=1, w_end=0.7,
                         w_start_reg=0.5, w_end_reg=0.3, w_cls=1.3)
    tw = {"label_weights": torch.tensor([1.0, 2.0, 0.5, 1.5, 3.0])} if label_weights else None
    return build_loss(lp, tw)


def _uneven_micro_batches(ignore_cls=False):
    """Two micro-batches collated at their own lengths (32 and 24 tokens), with ignored spans and (focal, whose
    ignore_index is -1) one ignored class target in the second micro-batch."""
    a = _with_ignored_spans(_batch(B=4, L=32, seed=4))
    b = _batch(B=4, L=24, seed=9)
    lb = dict(b[1])
    lb["start_class"] = lb["start_class"].clone() % 24
    lb["end_class"] = lb["end_class"].clone() % 24
    lb["start_class"][0] = -1
    if ignore_cls:
        lb["cls"] = lb["cls"].clone()
        lb["cls"][2] = -1
    return [a, (b[0], lb)]


@pytest.mark.parametrize("kind,lw", [("ce", False), ("ce", True), ("smooth", False), ("focal", False)])
def test_segmented_merge_equals_micro_batch_accumulation(kind, lw):
    """One merged pass over two unequal-length micro-batches (loss segments) gives the gradient and the loss of
    the reference's two accumulated micro-steps, to fp32 rounding."""
    from ml_recipe_distributed_pytorch_amd.data.collate import merge_micro_batches
    torch.manual_seed(0)
    model, _, _ = _build(3)
    loss_fn = _loss(kind, lw)
    mbs = _uneven_micro_batches(ignore_cls=kind == "focal")
    model.zero_grad()
    ref_loss = 0.0
    for inp, lab in mbs:
        loss = loss_fn(model(**inp), lab) / 2
        loss.backward()
        ref_loss += float(loss.detach())
    ref = model.store.grad.clone()
    model.zero_grad()
    inp, lab = merge_micro_batches(mbs, pad_token_id=0)
    assert inp["input_ids"].shape == (8, 32) and lab["segment_lengths"] == (32, 24)
    assert not bool(inp["attention_mask"][4:, 24:].any())
    loss = loss_fn(model(**inp), lab)
    loss.backward()
    got = model.store.grad.clone()
    assert float(loss.detach()) == pytest.approx(ref_loss, rel=1e-5)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-7)
    rec = loss_fn.last.to_floats()
    assert set(rec) >= {"start_class", "end_class", "start_reg", "end_reg", "cls", "loss"}


def test_engine_merge_segments_matches_accumulation():
    """TrainEngine(batch_split=1, merge_segments=2) consumes the two micro-batches, runs ONE pass and steps
    the optimizer with the accumulated reference gradient."""
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    torch.manual_seed(0)
    model, _, opt = _build(3)
    loss_fn = _loss("ce")
    mbs = _uneven_micro_batches()
    model.zero_grad()
    for inp, lab in mbs:
        (loss_fn(model(**inp), lab) / 2).backward()
    ref = model.store.grad.clone()
    eng = TrainEngine(model, loss_fn, opt, batch_split=1, merge_segments=2, max_grad_norm=0.0)
    seen = {}
    orig = opt.step

    def spy(**kw):
        seen["g"] = model.store.grad.clone()
        return orig(**kw)
    opt.step = spy
    model.zero_grad()
    calls = []
    orig_fwd = model.forward
    model.forward = lambda *a, **k: (calls.append(1), orig_fwd(*a, **k))[1]
    eng.step(mbs)
    assert len(calls) == 1
    torch.testing.assert_close(seen["g"], ref, rtol=1e-5, atol=1e-7)


def test_plan_exact_merge():
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.train.memory import plan_exact_merge
    cfg = get_config("bert-base-uncased")
    # the reference's 128 x 2 at seq 512: one pass of 128 segments on 288 GB
    assert plan_exact_merge(cfg, 512, 256, 288 * 2**30, requested=128) == (128, 128)
    # a small device: passes of as many micro-batches as fit, the split untouched
    split, G = plan_exact_merge(cfg, 512, 256, 24 * 2**30, requested=128)
    assert split == 128 and 1 <= G < 128 and 128 % G == 0
    # a micro-batch that does not fit raises the split, nothing merged
    split, G = plan_exact_merge(cfg, 512, 256, 24 * 2**30, requested=1)
    assert split > 1 and G == 1
