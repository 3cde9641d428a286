"""HIP-graph replay of the training step (TrainEngine(graph=True)) against the eager step: same batches,
same dropout seeds (host-drawn, written to the model's device seed word before each replay), so losses and
weights must agree bit for bit.  Covered: one micro-batch
per step; gradient accumulation (first / middle / last micro-batch graphs); the native RCCL reducer's bucket
all-reduces captured inside the boundary graph (forced 1-rank communicator); and the reference-heads path,
which must stay eager (its classifier dropout key is drawn on the host)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(cuda, graph, steps=5, B=2, L=512, split=1, reducer=False, lengths=None, stats=None):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.parallel.reducer import GradReducer
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    cfg = get_config("bert-base-uncased", num_hidden_layers=2)
    model = BertForQuestionAnswering(cfg, seed=5).to(cuda).train()
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=1e-4, eps=1e-6,
                     correct_bias=False, zero_grad_fn=model.zero_grad)
    red = GradReducer(model, bucket_cap_mb=8, force=True) if reducer else None
    eng = TrainEngine(model, build_loss(lp), opt, max_grad_norm=1.0, graph=graph, batch_split=split, reducer=red)
    torch.manual_seed(77)   # the per-micro-step dropout seeds
    losses = []
    for i in range(steps):
        mbs = []
        for j in range(split):
            Li = lengths[i % len(lengths)] if lengths else L
            inputs, labels = synth_batch_native(B, Li, 64, SpecialIds(), seed=10 + i * split + j)
            mbs.append((to_device(inputs, cuda), to_device(labels, cuda)))
        res = eng.step(mbs)
        losses.append(res.losses["loss"].item())
    torch.cuda.synchronize()
    master = model.store.master.clone()
    replays = eng.graph_replays
    kinds = sorted((k[1], k[2]) for k in eng._graphs)
    if stats is not None:
        stats.update(shapes=len(eng._graph_shapes), graphs=len(eng._graphs), eager=eng.graph_eager_steps,
                     pools={g.pool() for g, _, _, _ in eng._graphs.values()})
    eng.release_graph()
    if red is not None:
        red.close()
    return losses, master, replays, model, kinds


def _same(model, le, me, lg, mg):
    """Every kernel of the step is deterministic (the embedding backward sums each word's rows in a fixed order
    since round 5): graph replay and eager must agree bit for bit."""
    for a, b in zip(le, lg):
        assert a == b, (a, b)
    diff = int((mg != me).sum())
    assert diff == 0, f"{diff} of {me.numel()} master weights differ between graph replay and eager"


def test_graph_replay_matches_eager(cuda):
    le, me, r0, model, _ = _run(cuda, graph=False)
    lg, mg, r1, _, kinds = _run(cuda, graph=True)
    assert r0 == 0 and r1 == 3          # two eager warm-up steps, then capture + 3 replays
    assert kinds == [(True, False)]
    _same(model, le, me, lg, mg)


def test_graph_replay_with_accumulation(cuda):
    """batch_split 4: the first micro-batch overwrites the arena (and refreshes Wᵀ in its graph), the middle
    ones and the last accumulate — three graphs, replayed 4 × 4 − 2 times."""
    le, me, _, model, _ = _run(cuda, graph=False, steps=4, split=4)
    lg, mg, r1, _, kinds = _run(cuda, graph=True, steps=4, split=4)
    assert r1 == 14 and kinds == [(False, False), (True, False)]
    _same(model, le, me, lg, mg)


def test_graph_replay_with_reducer_and_accumulation(cuda):
    """The forced 1-rank native RCCL reducer: its bucket all-reduces (fence → ncclAllReduce on the comm
    stream → join) are captured in the boundary micro-batch's graph; averaging over one rank is the identity,
    so graph + reducer must equal eager without a reducer."""
    le, me, _, model, _ = _run(cuda, graph=False, steps=4, split=3)
    lg, mg, r1, _, kinds = _run(cuda, graph=True, steps=4, split=3, reducer=True)
    assert r1 == 10 and kinds == [(False, False), (False, True), (True, False)]
    _same(model, le, me, lg, mg)


def test_graph_not_used_with_reference_heads(cuda, monkeypatch):
    """HQ_FUSED_HEADS=0: the autograd heads draw their classifier-dropout key on the host, so a graph would
    freeze one mask — the engine must stay eager and match the plain eager run."""
    monkeypatch.setenv("HQ_FUSED_HEADS", "0")
    le, me, _, model, _ = _run(cuda, graph=False, steps=3)
    lg, mg, r1, _, _ = _run(cuda, graph=True, steps=3)
    assert r1 == 0
    _same(model, le, me, lg, mg)


def test_graph_shape_cap_runs_other_lengths_eagerly(cuda):
    """Padded NQ batches vary in length: graphs are captured for the first two shapes only (one shared
    mempool), every other length runs eagerly beside them, and the result still equals the eager run."""
    Ls = [512, 256, 384, 512, 256, 384, 128]
    le, me, _, model, _ = _run(cuda, graph=False, steps=7, lengths=Ls)
    st = {}
    lg, mg, r1, _, kinds = _run(cuda, graph=True, steps=7, lengths=Ls, stats=st)
    # steps 1-2 eager warm-up; 384 and 512 captured (steps 3, 4) and replayed (step 6); 256, 128 eager (5, 7)
    assert r1 == 3 and st["shapes"] == 2 and st["graphs"] == 2 and st["eager"] == 2, st
    assert len(st["pools"]) == 1, st
    _same(model, le, me, lg, mg)


def test_graph_replay_matches_eager_under_per_op_sync(cuda, monkeypatch):
    """Regression (profiles/r6_debug_asserts): with a device synchronisation after every kernel op (the debug
    build's proxy, here over the release kernels), the replays diverged from eager at the third replay while a
    runtime hipMemsetAsync (the embedding gradients' fresh zero-fill) sat inside the captured step as a memset
    node.  The step graph now holds kernel nodes only; replay must equal eager bit for bit under any timing."""
    monkeypatch.setenv("HQ_SYNC_PROXY", "1")
    le, me, _, model, _ = _run(cuda, graph=False)
    lg, mg, r1, _, _ = _run(cuda, graph=True)
    assert r1 == 3
    _same(model, le, me, lg, mg)


@pytest.mark.gpu
def test_prefetched_batches_match_direct_copies(cuda):
    """DevicePrefetcher (copy stream, one batch ahead): a training run fed through prefetch_to_device ends with the
    same weights and losses as one fed by plain to_device copies on the compute stream."""
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, prefetch_to_device, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    cfg = get_config("bert-base-uncased", num_hidden_layers=2)
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, w_start=1, w_end=1, w_start_reg=1, w_end_reg=1, w_cls=1)
    host = [tuple(synth_batch_native(16, 128, 32, SpecialIds(), seed=s)) for s in range(6)]
    runs = {}
    for pf in (False, True):
        torch.manual_seed(0)   # the host dropout seeds
        m = BertForQuestionAnswering(cfg, seed=0).to(cuda).train()
        opt = FusedAdamW(optimizer_groups(m.named_parameters(), 1e-4), m.store, lr=1e-4, correct_bias=False,
                         zero_grad_fn=m.zero_grad)
        eng = TrainEngine(m, build_loss(lp), opt)
        feed = prefetch_to_device(host, cuda) if pf else (to_device(b, cuda) for b in host)
        losses = [eng.step([(x, y)]).losses.to_floats()["loss"] for x, y in feed]
        torch.cuda.synchronize()
        runs[pf] = (losses, m.store.master.clone())
    assert runs[False][0] == runs[True][0]
    assert torch.equal(runs[False][1], runs[True][1])
