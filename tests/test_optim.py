"""Arena optimizers vs textbook per-parameter formulas (HF AdamW, reference AdaMod), clipping, schedule,
optimizer state round trip."""
import math

import pytest
import torch

from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
from ml_recipe_distributed_pytorch_amd.models.config import get_config
from ml_recipe_distributed_pytorch_amd.train.optim import (FusedAdaMod, FusedAdamW, get_linear_schedule_with_warmup,
                                                           grad_norm_and_clip)
from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups


def _model():
    return BertForQuestionAnswering(get_config("bert-tiny-test"), precision="fp32", seed=0)


def _hf_adamw(params, grads, state, lr, wd, b1, b2, eps, correct_bias, step):
    for i, (p, g) in enumerate(zip(params, grads)):
        m, v = state.setdefault(i, (torch.zeros_like(p), torch.zeros_like(p)))
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = v.sqrt().add_(eps)
        ss = lr * math.sqrt(1 - b2 ** step) / (1 - b1 ** step) if correct_bias else lr
        p.addcdiv_(m, denom, value=-ss)
        if wd[i] > 0:
            p.add_(p, alpha=-lr * wd[i])


def _adamod(params, grads, state, lr, wd, b1, b2, b3, eps, step):
    for i, (p, g) in enumerate(zip(params, grads)):
        m, v, n = state.setdefault(i, (torch.zeros_like(p), torch.zeros_like(p), torch.zeros_like(p)))
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = v.sqrt().add_(eps)
        ss = lr * math.sqrt(1 - b2 ** step) / (1 - b1 ** step)
        if wd[i] != 0:
            p.add_(p, alpha=-wd[i] * lr)
        ss = torch.full_like(denom, ss) / denom
        n.mul_(b3).add_(ss, alpha=1 - b3)
        p.add_(-torch.minimum(ss, n) * m)


@pytest.mark.parametrize("kind,correct_bias", [("adamw", False), ("adamw", True), ("adamod", None)])
def test_arena_optimizer_matches_formula(kind, correct_bias):
    torch.manual_seed(0)
    m = _model()
    named = list(m.named_parameters())
    groups = optimizer_groups(named, 0.01)
    if kind == "adamw":
        opt = FusedAdamW(groups, m.store, lr=1e-3, eps=1e-6, correct_bias=correct_bias)
    else:
        opt = FusedAdaMod(groups, m.store, lr=1e-3)
    wd = {id(p): g["weight_decay"] for g in groups for p in g["params"]}
    params = [p.detach().clone() for _, p in named]
    wds = [wd[id(p)] for _, p in named]
    state = {}
    for step in range(1, 4):
        grads = [torch.randn_like(p) for p in params]
        for (_, p), g in zip(named, grads):
            p.grad.copy_(g)
        opt.step()
        if kind == "adamw":
            _hf_adamw(params, grads, state, 1e-3, wds, 0.9, 0.999, 1e-6, correct_bias, step)
        else:
            _adamod(params, grads, state, 1e-3, wds, 0.9, 0.999, 0.999, 1e-8, step)
    for (n, p), q in zip(named, params):
        torch.testing.assert_close(p.detach(), q, atol=1e-6, rtol=1e-5, msg=n)


def test_no_decay_groups():
    m = _model()
    groups = optimizer_groups(list(m.named_parameters()), 0.01)
    names = {id(p): n for n, p in m.named_parameters()}
    for g in groups:
        for p in g["params"]:
            n = names[id(p)]
            assert (g["weight_decay"] == 0.0) == ("bias" in n or "LayerNorm.weight" in n), n


def test_clip_matches_torch():
    m = _model()
    torch.manual_seed(1)
    for p in m.parameters():
        p.grad.copy_(torch.randn_like(p) * 3)
    ref = [p.grad.clone() for p in m.parameters()]
    norm, coef = grad_norm_and_clip(m.store, 1.0)
    tot = torch.sqrt(sum((r.double() ** 2).sum() for r in ref))
    assert abs(norm.item() - tot.item()) / tot.item() < 1e-5
    assert abs(coef.item() - 1.0 / (tot.item() + 1e-6)) < 1e-6


def test_clip_coef_applied_in_step():
    m1, m2 = _model(), _model()
    torch.manual_seed(2)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        g = torch.randn_like(p1) * 5
        p1.grad.copy_(g)
        p2.grad.copy_(g)
    o1 = FusedAdamW(optimizer_groups(list(m1.named_parameters()), 0.01), m1.store, lr=1e-3)
    o2 = FusedAdamW(optimizer_groups(list(m2.named_parameters()), 0.01), m2.store, lr=1e-3)
    _, coef = grad_norm_and_clip(m1.store, 1.0)
    o1.step(clip_coef=coef)
    torch.nn.utils.clip_grad_norm_(list(m2.parameters()), 1.0)
    o2.step()
    torch.testing.assert_close(m1.store.master, m2.store.master, atol=1e-6, rtol=1e-5)


def test_linear_warmup_schedule():
    m = _model()
    opt = FusedAdamW(optimizer_groups(list(m.named_parameters()), 0.0), m.store, lr=1.0)
    sch = get_linear_schedule_with_warmup(opt, 4, 10)
    lrs = []
    for _ in range(11):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert lrs[:5] == [0.0, 0.25, 0.5, 0.75, 1.0]
    assert abs(lrs[7] - 0.5) < 1e-9 and lrs[10] == 0.0


def test_optimizer_state_roundtrip(tmp_path):
    m = _model()
    opt = FusedAdamW(optimizer_groups(list(m.named_parameters()), 0.01), m.store, lr=1e-3)
    for p in m.parameters():
        p.grad.normal_()
    opt.step()
    sd = opt.state_dict()
    path = tmp_path / "o.pt"
    torch.save(sd, path)
    m2 = _model()
    m2.load_state_dict(m.state_dict())
    opt2 = FusedAdamW(optimizer_groups(list(m2.named_parameters()), 0.01), m2.store, lr=1e-3)
    opt2.load_state_dict(torch.load(path, weights_only=True))
    torch.testing.assert_close(opt2._arenas["exp_avg"], opt._arenas["exp_avg"])
    torch.testing.assert_close(opt2._arenas["exp_avg_sq"], opt._arenas["exp_avg_sq"])
    for p1, p2 in zip(m.parameters(), m2.parameters()):
        g = torch.randn_like(p1)
        p1.grad.copy_(g)
        p2.grad.copy_(g)
    opt.step()
    opt2.step()
    torch.testing.assert_close(m.store.master, m2.store.master)
    # per-parameter state layout matches torch/HF optimizers (step, exp_avg, exp_avg_sq)
    st0 = sd["state"][0]
    assert set(st0) == {"step", "exp_avg", "exp_avg_sq"}
