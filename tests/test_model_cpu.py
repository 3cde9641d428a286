"""Fused BERT/RoBERTa QA model (CPU path) vs HF transformers + the reference heads; state-dict layout."""
import copy

import pytest
import torch
import torch.nn as nn

from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering, load_pretrained
from ml_recipe_distributed_pytorch_amd.models.config import get_config

transformers = pytest.importorskip("transformers")

TINY = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256)


def _hf_model(cfg):
    kw = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, num_hidden_layers=cfg.num_hidden_layers,
              num_attention_heads=cfg.num_attention_heads, intermediate_size=cfg.intermediate_size,
              max_position_embeddings=cfg.max_position_embeddings, type_vocab_size=cfg.type_vocab_size,
              hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, layer_norm_eps=cfg.layer_norm_eps,
              pad_token_id=cfg.pad_token_id)
    if cfg.family == "roberta":
        hc = transformers.RobertaConfig(**kw)
        hc._attn_implementation = "eager"
        enc = transformers.RobertaModel(hc)
    else:
        hc = transformers.BertConfig(**kw)
        hc._attn_implementation = "eager"
        enc = transformers.BertModel(hc)
    H = cfg.hidden_size

    class QA(nn.Module):
        def __init__(self):
            super().__init__()
            self.transformer = enc
            self.position_outputs = nn.Linear(H, 2)
            self.classifier = nn.Sequential(nn.Dropout(0.0), nn.Linear(H, 5))
            self.reg_start = nn.Sequential(nn.Linear(H, 1), nn.Sigmoid())
            self.reg_end = nn.Sequential(nn.Linear(H, 1), nn.Sigmoid())

        def forward(self, input_ids, attention_mask, token_type_ids):
            out = self.transformer(input_ids=input_ids, attention_mask=attention_mask, token_type_ids=token_type_ids)
            seq, pooled = out[0], out[1]
            s, e = self.position_outputs(seq).split(1, dim=-1)
            return {"start_class": s.squeeze(-1), "end_class": e.squeeze(-1), "cls": self.classifier(pooled),
                    "start_reg": self.reg_start(pooled).squeeze(-1), "end_reg": self.reg_end(pooled).squeeze(-1)}

    return QA()


def _pair(name, **over):
    cfg = get_config(name, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, **over)
    ours = BertForQuestionAnswering(cfg, precision="fp32", seed=3)
    ref = _hf_model(cfg)
    sd = {k: v for k, v in ours.state_dict().items()}
    missing, unexpected = ref.load_state_dict(sd, strict=False)
    assert not [k for k in missing if "position_ids" not in k], missing
    assert not [k for k in unexpected if "position_ids" not in k], unexpected
    return cfg, ours, ref


def _batch(cfg, B=3, L=24, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(5, cfg.vocab_size, (B, L), generator=g)
    ids[1, 17:] = cfg.pad_token_id
    mask = (ids != cfg.pad_token_id).long()
    tt = torch.zeros_like(ids)
    if cfg.type_vocab_size > 1:
        tt[:, 9:] = 1
    return ids, mask, tt


@pytest.mark.parametrize("name,over", [("bert-tiny-test", {}), ("roberta-base", dict(vocab_size=1000, **TINY))])
def test_forward_backward_parity_with_hf(name, over):
    cfg, ours, ref = _pair(name, **over)
    ids, mask, tt = _batch(cfg)
    ours.train()
    ref.train()
    a = ours(ids, mask, tt)
    b = ref(ids, mask, tt)
    for k in a:
        torch.testing.assert_close(a[k], b[k], atol=2e-5, rtol=1e-4, msg=k)
    w = {k: torch.randn_like(v) for k, v in a.items()}
    sum((a[k] * w[k]).sum() for k in a).backward()
    sum((b[k] * w[k]).sum() for k in b).backward()
    rp = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        assert n in rp, n
        torch.testing.assert_close(p.grad, rp[n].grad, atol=5e-5, rtol=1e-3, msg=n)


def test_dropout_train_vs_eval():
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    ids, mask, tt = _batch(cfg)
    m.eval()
    e1, e2 = m(ids, mask, tt), m(ids, mask, tt)
    torch.testing.assert_close(e1["start_class"], e2["start_class"])
    m.train()
    torch.manual_seed(0)
    t1 = m(ids, mask, tt)
    assert not torch.allclose(t1["start_class"], e1["start_class"])


def test_state_dict_hf_names_and_roundtrip(tmp_path):
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    sd = m.state_dict()
    for k in ("transformer.embeddings.word_embeddings.weight", "transformer.encoder.layer.1.attention.self.key.bias",
              "transformer.encoder.layer.0.output.LayerNorm.weight", "transformer.pooler.dense.weight",
              "position_outputs.weight", "classifier.1.weight", "reg_start.0.bias", "reg_end.0.weight",
              "transformer.embeddings.position_ids"):
        assert k in sd, k
    assert not any(".qkv." in k for k in sd)
    path = tmp_path / "m.ch"
    torch.save({"model": sd}, path)
    m2 = BertForQuestionAnswering(cfg, precision="fp32", seed=2)
    m2.load_state_dict(torch.load(path, weights_only=True)["model"])
    ids, mask, tt = _batch(cfg)
    m.eval(), m2.eval()
    torch.testing.assert_close(m(ids, mask, tt)["cls"], m2(ids, mask, tt)["cls"])
    # fused QKV arena entry is the concatenation of the HF q/k/v views
    p = "transformer.encoder.layer.0.attention.self."
    qkv = m.store.view("transformer.encoder.layer.0.qkv.weight", "master")
    torch.testing.assert_close(qkv, torch.cat([sd[p + "query.weight"], sd[p + "key.weight"], sd[p + "value.weight"]]))


def test_load_pretrained_prefixes(tmp_path):
    from safetensors.torch import save_file
    cfg = get_config("bert-tiny-test")
    src = BertForQuestionAnswering(cfg, precision="fp32", seed=5)
    enc = {"bert." + k[len("transformer."):]: v.contiguous() for k, v in src.state_dict().items()
           if k.startswith("transformer.") and "position_ids" not in k}
    save_file(enc, str(tmp_path / "model.safetensors"))
    dst = BertForQuestionAnswering(cfg, precision="fp32", seed=6)
    load_pretrained(dst, str(tmp_path))
    for k, v in src.state_dict().items():
        if k.startswith("transformer."):
            torch.testing.assert_close(dst.state_dict()[k], v, msg=k)


def test_deepcopy_keeps_arena_views():
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    c = copy.deepcopy(m)
    p = dict(c.named_parameters())["transformer.encoder.layer.0.attention.self.query.weight"]
    assert p.data_ptr() >= c.store.master.data_ptr()
    assert p.data_ptr() < c.store.master.data_ptr() + c.store.master.numel() * 4
    torch.testing.assert_close(c.store.master, m.store.master)


def test_grad_accumulation_and_zero_grad():
    cfg = get_config("bert-tiny-test", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    ids, mask, tt = _batch(cfg)
    m.train()
    m.zero_grad()
    m(ids, mask, tt)["cls"].sum().backward()
    g1 = m.store.grad.clone()
    m(ids, mask, tt)["cls"].sum().backward()
    torch.testing.assert_close(m.store.grad, 2 * g1, atol=1e-5, rtol=1e-5)
    m.zero_grad()
    m(ids, mask, tt)["cls"].sum().backward()
    torch.testing.assert_close(m.store.grad, g1, atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("shape", ["layers", "heads"])
def test_head_mask_scales_each_heads_context(shape):
    """head_mask (reference model.py:43-48; HF multiplies head h's attention probabilities by m_h): the output
    equals the unmasked model with the out-projection columns of head h scaled by m_h, a zero head passes no
    gradient into its Q/K/V, and the mask [nh] applies to every layer.  (transformers 5.x dropped head_mask,
    so the oracle is that algebraic identity.)"""
    cfg = get_config("bert-tiny-test", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    nh, NL, dh = cfg.num_attention_heads, cfg.num_hidden_layers, cfg.head_dim
    a = BertForQuestionAnswering(cfg, precision="fp32", seed=3)
    b = copy.deepcopy(a)
    if shape == "layers":
        hm = torch.rand(NL, nh) * 2
        hm[0, 0] = 0.0
    else:
        hm = torch.rand(nh) * 2
        hm[0] = 0.0
    full = hm if hm.dim() == 2 else hm.unsqueeze(0).expand(NL, nh)
    cols = full.repeat_interleave(dh, dim=1)
    with torch.no_grad():
        for i in range(NL):
            b.store.params[f"transformer.encoder.layer.{i}.attention.output.dense.weight"].mul_(cols[i])
    b.store.mark_master_dirty()
    ids, mask, tt = _batch(cfg)
    oa = a(ids, mask, tt, head_mask=hm)
    ob = b(ids, mask, tt)
    for k in oa:
        torch.testing.assert_close(oa[k], ob[k], atol=1e-5, rtol=1e-4, msg=k)
    w = {k: torch.randn_like(v) for k, v in oa.items()}
    sum((oa[k] * w[k]).sum() for k in oa).backward()
    sum((ob[k] * w[k]).sum() for k in ob).backward()
    pb = dict(b.named_parameters())
    for n, p in a.named_parameters():
        g = pb[n].grad
        if n.endswith("attention.output.dense.weight"):
            g = g * cols[int(n.split(".")[3])]
        torch.testing.assert_close(p.grad, g, atol=1e-5, rtol=1e-4, msg=n)
    # the zero head of layer 0 gets no gradient in its query / key / value rows
    q = a.store.params["transformer.encoder.layer.0.attention.self.query.weight"].grad
    assert float(q[:dh].abs().max()) == 0.0 and float(q[dh:].abs().max()) > 0.0
    # all-ones is the unmasked model
    torch.testing.assert_close(a(ids, mask, tt, head_mask=torch.ones(nh))["start_class"],
                               a(ids, mask, tt)["start_class"])


def test_ln_from_y_guard_flags():
    """The LayerNorm-from-y guard: a LayerNorm whose weights have a column with γ = 0 or |β| > 8·|γ| (typical of
    pretrained checkpoints' small-γ columns) stores z; random-init weights never trip it; loading new weights
    re-runs it."""
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    assert [m.ln_from_y_ok(i, w) for i in range(2) for w in (0, 1)] == [True] * 4
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["transformer.encoder.layer.1.attention.output.LayerNorm.weight"][7] = 1e-3
    sd["transformer.encoder.layer.1.attention.output.LayerNorm.bias"][7] = 0.5
    sd["transformer.encoder.layer.0.output.LayerNorm.weight"][3] = 0.0
    m.load_state_dict(sd)
    assert [m.ln_from_y_ok(i, w) for i in range(2) for w in (0, 1)] == [True, False, False, True]
    with torch.no_grad():   # an optimizer moving the weights back: refresh reports the change
        m.store.params["transformer.encoder.layer.1.attention.output.LayerNorm.bias"][7] = 0.005
    assert m.refresh_ln_modes() is True and m.ln_from_y_ok(1, 0)


def test_finetune_module_train_modes():
    """Reference finetune mode (init.py:86-92, trainer.py:227-234): model.eval() and .train() on the trainable
    modules only — the encoder's dropout follows `transformer`, the classifier dropout follows `classifier`."""
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    ids, mask, tt = _batch(cfg)
    m.eval()
    ref = m(ids, mask, tt)
    m.classifier.train()   # finetune_class only: encoder deterministic, classifier dropout on
    torch.manual_seed(0)
    a = m(ids, mask, tt)
    torch.testing.assert_close(a["start_class"], ref["start_class"])
    assert not torch.allclose(a["cls"], ref["cls"])
    m.eval()
    m.transformer.train()  # finetune_transformer: encoder dropout on
    torch.manual_seed(0)
    b = m(ids, mask, tt)
    assert not torch.allclose(b["start_class"], ref["start_class"])


def test_ln_guard_load_state_dict_bumps_version():
    """load_state_dict re-runs the LayerNorm-from-y guard eagerly (never inside a later graph capture) and bumps
    ``ln_mode_version``, which a TrainEngine compares before every pass to release stale graphs."""
    cfg = get_config("bert-tiny-test")
    m = BertForQuestionAnswering(cfg, precision="fp32", seed=1)
    v0 = getattr(m, "ln_mode_version", 0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["transformer.encoder.layer.0.output.LayerNorm.weight"][3] = 0.0
    m.load_state_dict(sd)
    assert m._ln_y is not None and m._ln_y[1] is False          # already evaluated, no lazy refresh pending
    assert m.ln_mode_version == v0 + 1


def test_engine_graph_key_includes_segment_lengths():
    """Two merged batches with the same padded length but different per-segment lengths must not share a
    captured graph: the module-path loss slices by the host tuple ``segment_lengths``, which a replay
    cannot refresh."""
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    ids = torch.zeros(4, 16, dtype=torch.int64)
    a = TrainEngine._shape_key({"input_ids": ids}, {"segments": torch.tensor([12, 16]), "segment_lengths": (12, 16)})
    b = TrainEngine._shape_key({"input_ids": ids}, {"segments": torch.tensor([16, 9]), "segment_lengths": (16, 9)})
    c = TrainEngine._shape_key({"input_ids": ids}, {"segments": torch.tensor([16, 9]), "segment_lengths": (16, 9)})
    assert a != b and b == c


def test_prefetch_to_device_cpu_yields_items_in_order():
    """The trainer's prefetcher on CPU: every item, in order, tensors equal to the source (plain to_device)."""
    import torch
    from ml_recipe_distributed_pytorch_amd.train.engine import prefetch_to_device
    items = [({"a": torch.arange(4) + i}, {"b": torch.ones(2) * i}) for i in range(5)]
    out = list(prefetch_to_device(items, "cpu"))
    assert len(out) == 5
    for i, (x, y) in enumerate(out):
        assert torch.equal(x["a"], torch.arange(4) + i) and torch.equal(y["b"], torch.ones(2) * i)
    assert list(prefetch_to_device([], "cpu")) == []
