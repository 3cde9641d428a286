"""Gradient accumulation semantics (reference ``trainer.py:197-204,284``): one optimizer step over
``batch_split`` micro-batches accumulates ∇(loss(micro) / batch_split) — the mean of per-micro-batch means.
With ignored spans (start/end class −1: CE averages over the VALID spans of each micro-batch) that is not the
gradient of the merged batch, which is why ``--auto_batch_split`` only merges micro-batches on request
('merge')."""
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


@pytest.mark.parametrize("val,expect", [(None, None), ("True", True), ("merge", "merge"), ("False", False)])
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
