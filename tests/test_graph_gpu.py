"""HIP-graph replay of the training step (TrainEngine(graph=True)) against the eager step: same batches,
same dropout seeds (host-drawn, written to the model's device seed word before each replay), so losses and
weights must agree (bitwise except the float-atomic embedding-gradient scatter)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(cuda, graph, steps=5, B=2, L=512):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    cfg = get_config("bert-base-uncased", num_hidden_layers=2)
    model = BertForQuestionAnswering(cfg, seed=5).to(cuda).train()
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=1e-4, eps=1e-6,
                     correct_bias=False, zero_grad_fn=model.zero_grad)
    eng = TrainEngine(model, build_loss(lp), opt, max_grad_norm=1.0, graph=graph)
    torch.manual_seed(77)   # the per-step dropout seeds
    losses = []
    for i in range(steps):
        inputs, labels = synth_batch_native(B, L, 64, SpecialIds(), seed=10 + i)
        res = eng.step([(to_device(inputs, cuda), to_device(labels, cuda))])
        losses.append(res.losses["loss"].item())
    torch.cuda.synchronize()
    master = model.store.master.clone()
    replays = eng.graph_replays
    eng.release_graph()
    return losses, master, replays, model


def test_graph_replay_matches_eager(cuda):
    le, me, r0, model = _run(cuda, graph=False)
    lg, mg, r1, _ = _run(cuda, graph=True)
    assert r0 == 0 and r1 == 3          # two eager warm-up steps, then capture + 3 replays
    for a, b in zip(le, lg):
        assert a == pytest.approx(b, rel=1e-5, abs=1e-6)
    atomic = torch.zeros_like(me, dtype=torch.bool)
    for e in model.store.entries:
        if "word_embeddings" in e.key or "position_embeddings" in e.key:
            atomic[e.offset:e.offset + e.numel] = True
    assert torch.equal(mg[~atomic], me[~atomic]) or torch.allclose(mg, me, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mg[atomic], me[atomic], rtol=1e-4, atol=1e-6)
