"""The exact-objective merge on the GPU (the trainer's default when auto_batch_split is unset): one fused pass
over two unequal-length micro-batches as loss segments (TrainEngine(batch_split=1, merge_segments=2)) must
reproduce the reference's accumulation of two micro-steps (TrainEngine(batch_split=2)) through the fused
encoder, the fused heads and the fused segment loss (reference ``trainer.py:197-204``: loss / batch_split per
micro-batch).  Dropout off, bf16.  The merged pass pads the shorter micro-batch with masked keys; per-row GEMMs
and LayerNorms are unchanged by that, so the two gradients differ only by the order of the wgrad sums over
tokens.  The graph-captured merged step must then equal the eager merged step (same key, replayed)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

LENGTHS = [(256, 192), (192, 256), (256, 192), (256, 192), (192, 256), (256, 192)]


def _setup(cuda, graph, batch_split, merge):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    cfg = get_config("bert-base-uncased", num_hidden_layers=2, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    model = BertForQuestionAnswering(cfg, seed=3).to(cuda).train()
    lp = SimpleNamespace(loss="ce", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=1e-4, eps=1e-6,
                     correct_bias=False, zero_grad_fn=model.zero_grad)
    eng = TrainEngine(model, build_loss(lp), opt, max_grad_norm=1.0, graph=graph, batch_split=batch_split,
                      merge_segments=merge)
    return model, opt, eng


def _micro_batches(cuda, step, lengths, B=4):
    """Two micro-batches collated at their own lengths; the first has 3 ignored spans (start/end class -1), so
    the per-segment valid-span normalisers differ (that is what makes a plain merge wrong)."""
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.train.engine import to_device
    mbs = []
    for j, L in enumerate(lengths):
        inputs, labels = synth_batch_native(B, L, 64, SpecialIds(), seed=100 + 2 * step + j)
        labels = dict(labels)
        if j == 0:
            for k in ("start_class", "end_class"):
                labels[k] = labels[k].clone()
                labels[k][1:] = -1
        mbs.append((to_device(inputs, cuda), to_device(labels, cuda)))
    return mbs


def _spy_grads(model, opt):
    seen = []
    orig = opt.step

    def spy(**kw):
        seen.append(model.store.grad.clone())
        return orig(**kw)
    opt.step = spy
    return seen


def test_merged_pass_matches_accumulated_micro_steps(cuda):
    ma, oa, ea = _setup(cuda, False, 2, 1)
    mm, om, em = _setup(cuda, False, 1, 2)
    p0 = ma.store.master.clone()
    assert torch.equal(p0, mm.store.master)
    ga, gm = _spy_grads(ma, oa), _spy_grads(mm, om)
    for step in range(3):
        mbs = _micro_batches(cuda, step, LENGTHS[step])
        la = 0.0
        for inp, lab in mbs:   # the reference objective: mean of the two micro-batch losses
            ea.micro_step(inp, lab)
            la += float(ea.loss_fn.last["loss"]) / 2
        lm = float(em.step(mbs).losses["loss"])
        assert la == pytest.approx(lm, rel=2e-3), (step, la, lm)
    torch.cuda.synchronize()
    assert len(ga) == len(gm) == 3
    for step, (a, m) in enumerate(zip(ga, gm)):
        assert torch.isfinite(m).all()
        rel = float((a - m).norm() / a.norm())
        assert rel < 1e-2, (step, rel)
    # parameters after three optimizer steps: the same trajectory (Adam normalises every element, so compare the
    # whole update vectors, not single elements whose gradient is rounding noise, e.g. the key bias)
    da, dm = ma.store.master - p0, mm.store.master - p0
    assert float((da - dm).norm() / da.norm()) < 0.1


def test_merged_graph_replay_matches_eager_merged(cuda):
    """Six merged steps whose micro-batch lengths alternate between (256, 192) and (192, 256): one padded
    length, two segment layouts, so two graph keys; captured after the warm-up and replayed."""
    me_model, _, ee = _setup(cuda, False, 1, 2)
    mg_model, _, eg = _setup(cuda, True, 1, 2)
    le, lg = [], []
    for step in range(len(LENGTHS)):
        mbs = _micro_batches(cuda, step, LENGTHS[step])
        le.append(float(ee.step(mbs).losses["loss"]))
        lg.append(float(eg.step(mbs).losses["loss"]))
    torch.cuda.synchronize()
    replays = eg.graph_replays
    keys = len(eg._graphs)
    eg.release_graph()
    assert replays >= 1 and keys == 2, (replays, keys)
    for a, b in zip(le, lg):
        assert a == b, (a, b)
    me, mg = me_model.store.master, mg_model.store.master
    assert int((mg != me).sum()) == 0   # every kernel deterministic: graph replay == eager bit for bit
