"""Fused QA heads + losses (csrc/kernels/heads.hip) against the fp32 PyTorch reference path
(``models.heads.reference_heads`` + the ``WeightedLoss`` modules) on the same bf16 encoder output, the same
master weights and the same classifier-dropout mask (counter-hash RNG).

Forward outputs, the five loss terms and the total, and the backward (every head weight / bias gradient
in the arena and d seq) are compared for the three class losses (CE with class weights, focal, label
smoothing), ragged batches (B not a multiple of the 32-sample tile), ignored span targets, the
``1/batch_split`` scaling, accumulation into the arena and the general path (gradients that did not come
from the fused loss)."""
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("start_class", "end_class", "start_reg", "end_reg", "cls")


def _model(cuda, H=768, NL=5, p=0.1):
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    cfg = get_config("bert-base-uncased", num_hidden_layers=1, hidden_size=H, num_attention_heads=H // 64,
                     intermediate_size=4 * H, num_labels=NL, hidden_dropout_prob=p)
    m = BertForQuestionAnswering(cfg, seed=3).to(cuda).train()
    with torch.no_grad():  # non-trivial biases so every bias path is exercised
        for k in ("transformer.pooler.dense.bias", "classifier.1.bias", "reg_start.0.bias", "reg_end.0.bias",
                  "position_outputs.bias"):
            m.store.params[k].uniform_(-0.5, 0.5)
    return m


def _loss(kind, NL=5, label_weights=False):
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    lp = SimpleNamespace(loss=kind, smooth_alpha=0.1, focal_alpha=0.7, focal_gamma=2.0, w_start=1.0, w_end=0.5,
                         w_start_reg=2.0, w_end_reg=1.5, w_cls=0.8)
    tw = {"label_weights": torch.linspace(0.5, 2.0, NL)} if label_weights else None
    return build_loss(lp, tw, n_classes=NL).to(torch.device("cuda", 0))


def _targets(cuda, B, L, NL, seed=0):
    g = torch.Generator().manual_seed(seed)
    s = torch.randint(0, L, (B,), generator=g)
    e = torch.randint(0, L, (B,), generator=g)
    s[::5] = -1  # ignored spans
    e[1::7] = -1
    c = torch.randint(0, NL, (B,), generator=g)
    return {"start_class": s.to(cuda), "end_class": e.to(cuda), "start_reg": torch.rand(B, generator=g).to(cuda),
            "end_reg": torch.rand(B, generator=g).to(cuda), "cls": c.to(cuda)}


def _head_grads(m):
    from ml_recipe_distributed_pytorch_amd.models.heads import _W_KEYS
    return {k: m.store.view(k, "grad").clone() for k in _W_KEYS}


def _run(m, seq0, targets, loss_fn, fused, seed=1234, scale=1.0 / 3):
    from ml_recipe_distributed_pytorch_amd.models.heads import fused_heads, reference_heads
    seq = seq0.detach().clone().requires_grad_(True)
    m.zero_grad()
    if not fused:
        m.store.grad.zero_()
        loss_fn._fused_cfg = None
    out = (fused_heads if fused else reference_heads)(m, seq, seed, True)
    assert (out.fused is not None) == fused
    total = loss_fn(out, targets)
    (total * scale).backward()
    torch.cuda.synchronize()
    return {k: out[k].detach().float() for k in KEYS}, dict(loss_fn.last.to_floats()), _head_grads(m), seq.grad.float()


def _close(a, b, what, rtol=2e-4, atol=2e-5):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol * (1 + b.abs().max().item()), msg=what)


@pytest.mark.parametrize("kind,lw,B,L,H", [("ce", False, 37, 50, 768), ("ce", True, 64, 128, 768),
                                           ("focal", False, 45, 64, 256), ("smooth", False, 33, 96, 1024),
                                           ("smooth", False, 256, 384, 768)])
def test_fused_heads_and_loss_match_reference(cuda, kind, lw, B, L, H):
    NL = 5
    m = _model(cuda, H=H, NL=NL)
    seq = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16)
    t = _targets(cuda, B, L, NL)
    of, lf, gf, df = _run(m, seq, t, _loss(kind, NL, lw), fused=True)
    orf, lr, gr, dr = _run(m, seq, t, _loss(kind, NL, lw), fused=False)
    for k in KEYS:
        _close(of[k], orf[k], "pred " + k)
    for k in lr:
        assert lf[k] == pytest.approx(lr[k], rel=2e-4, abs=1e-6), (k, lf[k], lr[k])
    for k in gr:
        _close(gf[k], gr[k], "grad " + k, rtol=1e-3, atol=1e-4)
    # d seq is bf16 on the fused path: compare at bf16 resolution
    _close(df, dr, "dseq", rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("kind,B,L,H", [("smooth", 37, 50, 768), ("ce", 16, 128, 1024)])
def test_fused_heads_fp32_sequence(cuda, kind, B, L, H):
    """--precision fp32: the fused head / loss kernels read an fp32 sequence and write an fp32 d seq (no ATen /
    vendor-BLAS head GEMMs in the fp32 step) — vs the reference heads on the same fp32 sequence."""
    NL = 5
    m = _model(cuda, H=H, NL=NL)
    seq = torch.randn(B, L, H, device=cuda) * 0.8
    t = _targets(cuda, B, L, NL)
    of, lf, gf, df = _run(m, seq, t, _loss(kind, NL), fused=True)
    orf, lr, gr, dr = _run(m, seq, t, _loss(kind, NL), fused=False)
    for k in KEYS:
        _close(of[k], orf[k], "pred " + k)
    for k in lr:
        assert lf[k] == pytest.approx(lr[k], rel=2e-4, abs=1e-6), (k, lf[k], lr[k])
    for k in gr:
        _close(gf[k], gr[k], "grad " + k, rtol=1e-3, atol=1e-4)
    _close(df, dr, "dseq", rtol=1e-4, atol=1e-5)   # fp32 d seq: no bf16 rounding now


@pytest.mark.parametrize("kind,lw,S,b,L", [("ce", True, 4, 8, 96), ("focal", False, 3, 11, 64),
                                           ("smooth", False, 128, 2, 512), ("ce", False, 2, 5, 40)])
def test_fused_loss_segments_match_reference(cuda, kind, lw, S, b, L):
    """Segment mode (exact-objective micro-batch merge): S segments of b samples with their own span lengths
    L_s <= L — the loss kernel against the CPU-oracle segmented WeightedLoss (span softmax cut at L_s, every term
    normalised per segment, averaged over segments)."""
    NL, H = 5, 768
    B = S * b
    m = _model(cuda, H=H, NL=NL)
    seq = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16)
    t = _targets(cuda, B, L, NL)
    g = torch.Generator().manual_seed(5)
    lens = [int(x) for x in torch.randint(L // 2, L + 1, (S,), generator=g)]
    lens[0] = L
    for s_ in range(S):   # each segment's targets lie inside its own length (or are ignored)
        for k in ("start_class", "end_class"):
            v = t[k][s_ * b:(s_ + 1) * b]
            v[v >= lens[s_]] = lens[s_] - 1
    if kind == "focal":
        t["cls"][3] = -1
    t["segments"] = torch.tensor(lens, dtype=torch.int32, device=cuda)
    t["segment_lengths"] = tuple(lens)
    of, lf, gf, df = _run(m, seq, t, _loss(kind, NL, lw), fused=True)
    orf, lr, gr, dr = _run(m, seq, t, _loss(kind, NL, lw), fused=False)
    for k in lr:
        assert lf[k] == pytest.approx(lr[k], rel=2e-4, abs=1e-6), (k, lf[k], lr[k])
    for k in gr:
        _close(gf[k], gr[k], "grad " + k, rtol=1e-3, atol=1e-4)
    _close(df, dr, "dseq", rtol=1e-2, atol=1e-2)


def test_fused_heads_general_gradient_path(cuda):
    """Gradients that do not come from the fused loss (a custom objective) take the packed path."""
    B, L, H, NL = 20, 40, 768, 5
    m = _model(cuda, H=H, NL=NL, p=0.0)
    seq0 = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16)
    from ml_recipe_distributed_pytorch_amd.models.heads import fused_heads, reference_heads
    res = []
    for fn in (fused_heads, reference_heads):
        seq = seq0.clone().requires_grad_(True)
        m.zero_grad()
        m.store.grad.zero_()
        out = fn(m, seq, 7, True)
        obj = (out["start_class"] ** 2).mean() + out["cls"][:, 1].sum() + out["end_reg"].sum()  # start_reg unused
        obj.backward()
        torch.cuda.synchronize()
        res.append((_head_grads(m), seq.grad.float()))
    for k in res[1][0]:
        _close(res[0][0][k], res[1][0][k], "grad " + k, rtol=1e-3, atol=1e-4)
    _close(res[0][1], res[1][1], "dseq", rtol=1e-2, atol=1e-2)


def test_fused_loss_plus_extra_term_scales_correctly(cuda):
    """fused loss × 1/3 + an extra objective on the same predictions: autograd sums the fused loss's unscaled
    buffers with the extra gradient, so the heads backward takes the general path and must add the missing
    (g − 1)·buffer (models/heads.py) — against the all-autograd reference heads + loss modules."""
    B, L, H, NL = 24, 48, 768, 5
    m = _model(cuda, H=H, NL=NL, p=0.0)
    seq0 = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16)
    t = _targets(cuda, B, L, NL)
    from ml_recipe_distributed_pytorch_amd.models.heads import fused_heads, reference_heads
    res = []
    for fused in (True, False):
        loss_fn = _loss("ce", NL)
        seq = seq0.clone().requires_grad_(True)
        m.zero_grad()
        if not fused:
            m.store.grad.zero_()
            loss_fn._fused_cfg = None
        out = (fused_heads if fused else reference_heads)(m, seq, 7, True)
        obj = loss_fn(out, t) / 3 + 0.25 * (out["start_class"] ** 2).mean() + out["cls"][:, 2].sum()
        obj.backward()
        torch.cuda.synchronize()
        res.append((_head_grads(m), seq.grad.float()))
    for k in res[1][0]:
        _close(res[0][0][k], res[1][0][k], "grad " + k, rtol=1e-3, atol=1e-4)
    _close(res[0][1], res[1][1], "dseq", rtol=1e-2, atol=1e-2)


def test_fused_heads_accumulate_and_eval(cuda):
    """Two micro-batches accumulate into the arena (no zero_grad between); eval uses p = 0 and the
    fused loss also runs under no_grad (validation)."""
    B, L, H, NL = 16, 32, 768, 5
    m = _model(cuda, H=H, NL=NL)
    seq = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16).requires_grad_(True)
    t = _targets(cuda, B, L, NL)
    loss_fn = _loss("ce", NL)
    from ml_recipe_distributed_pytorch_amd.models.heads import fused_heads
    m.zero_grad()
    loss_fn(fused_heads(m, seq, 5, True), t).backward()
    g1 = _head_grads(m)
    loss_fn(fused_heads(m, seq, 5, True), t).backward()
    g2 = _head_grads(m)
    for k in g1:
        _close(g2[k], 2 * g1[k], "accumulate " + k, rtol=1e-5, atol=1e-6)
    m.eval()
    with torch.no_grad():
        out = fused_heads(m, seq.detach(), 0, False)
        total = loss_fn(out, t)
    assert torch.isfinite(total).item() and loss_fn.last["loss"].item() == pytest.approx(total.item())


def test_fused_heads_with_frozen_heads(cuda):
    """finetune_class-style freezing (reference D16): the fused kernels still run; the frozen heads' arena
    gradients stay zero and the trainable classifier's match the autograd reference path."""
    B, L, H, NL = 16, 64, 768, 5
    m = _model(cuda, H=H, NL=NL, p=0.0)
    from ml_recipe_distributed_pytorch_amd.models.heads import _W_KEYS, fused_heads_possible
    for k in _W_KEYS:
        m.store.params[k].requires_grad_(k.startswith("classifier"))
    assert fused_heads_possible(m)
    seq = (torch.randn(B, L, H, device=cuda) * 0.8).to(torch.bfloat16)
    t = _targets(cuda, B, L, NL)
    of, lf, gf, _ = _run(m, seq, t, _loss("ce", NL), fused=True)
    orf, lr, gr, _ = _run(m, seq, t, _loss("ce", NL), fused=False)
    for k in _W_KEYS:
        if k.startswith("classifier"):
            _close(gf[k], gr[k], "grad " + k, rtol=1e-3, atol=1e-4)
        else:
            assert float(gf[k].abs().max()) == 0.0, k
