"""Whole-model parity: the HIP path (bf16) against the CPU reference path (fp32) of the same
weights, same inputs and the same dropout masks (shared counter-hash RNG)."""
import copy

import pytest
import torch

from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
from ml_recipe_distributed_pytorch_amd.models.config import get_config

pytestmark = pytest.mark.gpu


def _inputs(B, L, V):
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(1, V, (B, L), generator=g)
    ids[1, L - 5:] = 0
    tt = torch.zeros_like(ids)
    tt[:, L // 3:] = 1
    return ids, ids > 0, tt


@pytest.mark.parametrize("train,B,side", [(False, 3, False), (True, 3, False), (True, 4, False), (True, 3, True)])
def test_tiny_model_gpu_matches_cpu(cuda, train, B, side):
    """Every projection (fwd + GELU epilogue, dgrad, residual and GELU' epilogues on the transposed
    weight copies, split-K weight gradients at N, K = 128-multiples) runs on the own MFMA GEMMs;
    B = 3 gives M = 192 (128² tiles with an M tail), B = 4 M = 256."""
    _tiny_parity(cuda, train, B=B, side=side)


def test_head_mask_gpu_matches_cpu(cuda):
    """head_mask on the HIP path (masked context into the out-projection GEMM, masked dctx into the attention
    backward) against the CPU reference path of the same weights."""
    _tiny_parity(cuda, True, B=4, head_mask=torch.tensor([[0.0, 1.5], [1.0, 0.5]]))


def test_pretrained_like_layernorm_weights_gpu_matches_cpu(cuda, monkeypatch):
    """LayerNorm weights like a pretrained checkpoint's (γ log-uniform over [1e-3, 2], β ~ N(0, 0.5)): the
    from-y guard makes every such LayerNorm store z, so the HIP gradients match the fp32 exact-input reference
    at the usual tolerance.  Forcing the from-y backward on those weights shows what the guard prevents."""
    def ln_init(model):
        g = torch.Generator().manual_seed(3)
        with torch.no_grad():
            for n in model._ln_names():
                H = model.store.params[n + ".weight"].numel()
                model.store.params[n + ".weight"].copy_(torch.exp(torch.empty(H).uniform_(-6.9, 0.69, generator=g)))
                model.store.params[n + ".bias"].copy_(torch.randn(H, generator=g) * 0.5)
        model.store.mark_master_dirty()
        model._ln_y = None
    guarded = _tiny_parity(cuda, True, B=4, init=ln_init)
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering as M
    monkeypatch.setattr(M, "ln_from_y_ok", lambda self, i, w: True)
    forced = _tiny_parity(cuda, True, B=4, init=ln_init, check=False)
    assert guarded < 5e-2 and forced > guarded, (guarded, forced)


def _tiny_parity(cuda, train, B, side=False, head_mask=None, init=None, check=True):
    cfg = get_config("bert-tiny-test")
    cpu = BertForQuestionAnswering(cfg, seed=0)
    if init is not None:
        init(cpu)
    gpu = copy.deepcopy(cpu).to(cuda)
    if side:  # weight-grad GEMMs on the side stream (HQ_WGRAD_STREAM=1)
        gpu.grad_side_stream = torch.cuda.Stream(device=cuda)
    cpu.train(train)
    gpu.train(train)
    ids, mask, tt = _inputs(B, 64, cfg.vocab_size)
    torch.manual_seed(11)
    kw = {} if head_mask is None else {"head_mask": head_mask}
    oc = cpu(ids, mask, tt, **kw)
    torch.manual_seed(11)
    og = gpu(ids.to(cuda), mask.to(cuda), tt.to(cuda), **kw)
    for key in oc:
        a, b = og[key].float().cpu(), oc[key].float()  # classifier dropout: same counter-hash mask on both
        assert (a - b).abs().max().item() < 5e-2 * (1 + b.abs().max().item()), key
    # backward through both paths
    lc = sum(v.float().sum() for k, v in oc.items() if k != "cls")
    lg = sum(v.float().sum() for k, v in og.items() if k != "cls")
    cpu.zero_grad()
    gpu.zero_grad()
    lc.backward()
    lg.backward()
    if side:
        torch.cuda.current_stream().wait_stream(gpu.grad_side_stream)
    gc, gg = cpu.store.grad, gpu.store.grad.cpu()
    rel = (gc - gg).norm() / gc.norm()
    if check:
        assert rel.item() < 5e-2, f"grad arena rel err {rel.item():.3e}"
    return rel.item()


def test_bert_base_step_runs(cuda):
    cfg = get_config("bert-base-uncased")
    m = BertForQuestionAnswering(cfg, seed=0).to(cuda).train()
    ids, mask, tt = _inputs(2, 384, cfg.vocab_size)
    out = m(ids.to(cuda), mask.to(cuda), tt.to(cuda))
    loss = sum(v.float().mean() for v in out.values())
    m.zero_grad()
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(m.store.grad).all()
    assert m.store.grad.abs().sum().item() > 0


def test_bert_base_fp8_forward_close_to_bf16(cuda):
    """--precision fp8: forward projections on fp8 e4m3 operands stay close to the bf16 model."""
    cfg = get_config("bert-base-uncased", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForQuestionAnswering(cfg, seed=0).to(cuda).eval()
    ids, mask, tt = _inputs(4, 256, cfg.vocab_size)
    ids, mask, tt = ids.to(cuda), mask.to(cuda), tt.to(cuda)
    with torch.no_grad():
        ref = m(ids, mask, tt)
        m.set_precision("fp8")
        out = m(ids, mask, tt)
    for k in ("start_class", "end_class", "cls"):
        rel = ((out[k].float() - ref[k].float()).norm() / ref[k].float().norm()).item()
        assert rel < 0.1, (k, rel)
    m.train()
    loss = sum(v.float().mean() for v in m(ids, mask, tt).values())
    m.zero_grad()
    loss.backward()
    assert torch.isfinite(m.store.grad).all()


def test_memory_model_matches_measured_slope(cuda):
    """train/memory.py's per-sample bytes vs the measured growth of the fwd+bwd peak between two batch
    sizes (BERT-base, L = 256) — the model --auto_batch_split sizes micro-batches with."""
    from ml_recipe_distributed_pytorch_amd.train.memory import estimate
    cfg = get_config("bert-base-uncased")
    L = 256
    m = BertForQuestionAnswering(cfg, seed=0).to(cuda).train()
    peaks = {}
    for B in (8, 40):
        ids, mask, tt = _inputs(B, L, cfg.vocab_size)
        ids, mask, tt = ids.to(cuda), mask.to(cuda), tt.to(cuda)
        m.zero_grad()
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(cuda)
        base = torch.cuda.memory_allocated(cuda)
        loss = sum(v.float().mean() for v in m(ids, mask, tt).values())
        loss.backward()
        torch.cuda.synchronize()
        peaks[B] = torch.cuda.max_memory_allocated(cuda) - base
        del loss
    measured = (peaks[40] - peaks[8]) / 32
    est = estimate(cfg, L)
    modelled = est.act_bytes_per_sample + est.transient_bytes_per_sample
    assert measured == pytest.approx(modelled, rel=0.2), (measured, modelled)


def test_ln_guard_kernel_matches_cpu_rule(cuda):
    """The LayerNorm-from-y guard on the GPU is one own kernel (norm.hip ln_guard_kernel, no ATen chain) and gives
    the CPU rule's flags: γ = 0, |β| > 8·|γ| and a border case |β| = 8·|γ| (allowed)."""
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="bf16", seed=1).to(cuda)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["transformer.encoder.layer.1.attention.output.LayerNorm.weight"][7] = 1e-3
    sd["transformer.encoder.layer.1.attention.output.LayerNorm.bias"][7] = 0.5
    sd["transformer.encoder.layer.0.output.LayerNorm.weight"][3] = 0.0
    sd["transformer.encoder.layer.1.output.LayerNorm.weight"][5] = 0.25
    sd["transformer.encoder.layer.1.output.LayerNorm.bias"][5] = -2.0
    m.load_state_dict(sd)
    flags = m._ln_flags()
    assert flags.is_cuda and flags.dtype == torch.bool
    cpu = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    cpu.load_state_dict({k: v.cpu() for k, v in sd.items()})
    assert flags.cpu().tolist() == cpu._ln_flags().tolist() == [True, False, False, True]
