"""BERT / RoBERTa encoder + QA heads, MI355X-first.

Capability parity with the reference model (``modules/model/model/model.py:13-73``: HF
``BertModel``/``RobertaModel`` + ``position_outputs`` Linear(H,2), ``classifier`` Dropout+Linear(H,5),
``reg_start``/``reg_end`` Linear(H,1)+Sigmoid), re-designed around fused kernels:

* The encoder is a chain of ``torch.autograd.Function``s — one for the embeddings, one per
  encoder layer — each with an explicit backward.  Per layer forward = 4 own MFMA GEMMs with fused
  epilogues (QKV + bias, out-projection + bias, FFN1 + bias + GELU/GELU', FFN2 + bias) + flash attention
  + 2 residual/dropout/LayerNorm kernels; backward = 4 dgrad GEMMs (residual-add and GELU' epilogues),
  4 split-K weight-gradient GEMMs, the attention backward and 2 LayerNorm backwards.  Weight gradients
  are written straight into the fp32 grad arena and the layer then signals the gradient reducer, which
  overlaps its RCCL all-reduce with the rest of the backward (replaces DDP's per-parameter autograd
  hooks).
* Dropout: masks come from a counter hash (``ops.rng``, bit-identical in the HIP kernels).  The attention
  forward stores its keep-bits (1 bit per probability) for the backward; every other dropout site
  regenerates its mask from (seed, op id, element index) in the backward.
* Pooler + the four heads (``heads.py``): on the GPU one fused fp32 kernel each way plus one fused
  loss kernel (``csrc/kernels/heads.hip``); elsewhere ordinary fp32 autograd on the master parameters.
* ``state_dict()`` keys are the HF names under ``transformer.`` plus the reference head names, so
  reference checkpoints load and ours load into the reference (``embeddings.position_ids`` kept).
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional

import torch
import torch.nn as nn

from .. import ops
from .config import EncoderConfig
from .heads import fused_heads, fused_heads_available, reference_heads
from .params import Entry, ParamStore

LABELS = ["yes", "no", "short", "long", "unknown"]


# =========================================================================================== layout
def build_entries(cfg: EncoderConfig) -> List[Entry]:
    H, Fd, V, P, Tv = (cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size, cfg.max_position_embeddings,
                       cfg.type_vocab_size)
    NL = cfg.num_labels

    def lin(name, out_f, in_f, group, init="normal"):
        return [Entry(name + ".weight", (out_f, in_f), group, init, [(name + ".weight", 0, out_f)]),
                Entry(name + ".bias", (out_f,), group, "zeros" if init == "normal" else init,
                      [(name + ".bias", 0, out_f)])]

    def ln(name, group):
        return [Entry(name + ".weight", (H,), group, "ones", [(name + ".weight", 0, H)]),
                Entry(name + ".bias", (H,), group, "zeros", [(name + ".bias", 0, H)])]

    out: List[Entry] = []
    # QA heads (reference nn.Linear default init) + pooler: ready first in backward
    out += lin("position_outputs", 2, H, "head", "linear_default")
    out += lin("classifier.1", NL, H, "head", "linear_default")
    out += lin("reg_start.0", 1, H, "head", "linear_default")
    out += lin("reg_end.0", 1, H, "head", "linear_default")
    out += lin("transformer.pooler.dense", H, H, "head")
    for i in reversed(range(cfg.num_hidden_layers)):
        p = f"transformer.encoder.layer.{i}."
        g = f"layer.{i}"
        a = p + "attention.self."
        out.append(Entry(p + "qkv.weight", (3 * H, H), g, "normal",
                         [(a + "query.weight", 0, H), (a + "key.weight", H, 2 * H), (a + "value.weight", 2 * H, 3 * H)]))
        out.append(Entry(p + "qkv.bias", (3 * H,), g, "zeros",
                         [(a + "query.bias", 0, H), (a + "key.bias", H, 2 * H), (a + "value.bias", 2 * H, 3 * H)]))
        out += lin(p + "attention.output.dense", H, H, g)
        out += ln(p + "attention.output.LayerNorm", g)
        out += lin(p + "intermediate.dense", Fd, H, g)
        out += lin(p + "output.dense", H, Fd, g)
        out += ln(p + "output.LayerNorm", g)
    e = "transformer.embeddings."
    out += ln(e + "LayerNorm", "embeddings")
    out.append(Entry(e + "token_type_embeddings.weight", (Tv, H), "embeddings", "normal",
                     [(e + "token_type_embeddings.weight", 0, Tv)]))
    out.append(Entry(e + "position_embeddings.weight", (P, H), "embeddings", "normal",
                     [(e + "position_embeddings.weight", 0, P)]))
    out.append(Entry(e + "word_embeddings.weight", (V, H), "embeddings", "normal",
                     [(e + "word_embeddings.weight", 0, V)]))
    return out


def hf_param_order(cfg: EncoderConfig) -> List[str]:
    """``named_parameters()`` order of HF ``BertModel`` + the reference heads (``model.py:20-41``), so that
    optimizer-state indices line up with reference checkpoints."""
    e = "transformer.embeddings."
    names = [e + "word_embeddings.weight", e + "position_embeddings.weight", e + "token_type_embeddings.weight",
             e + "LayerNorm.weight", e + "LayerNorm.bias"]
    for i in range(cfg.num_hidden_layers):
        p = f"transformer.encoder.layer.{i}."
        for sub in ("attention.self.query", "attention.self.key", "attention.self.value", "attention.output.dense",
                    "attention.output.LayerNorm", "intermediate.dense", "output.dense", "output.LayerNorm"):
            names += [p + sub + ".weight", p + sub + ".bias"]
    names += ["transformer.pooler.dense.weight", "transformer.pooler.dense.bias"]
    for h in ("position_outputs", "classifier.1", "reg_start.0", "reg_end.0"):
        names += [h + ".weight", h + ".bias"]
    return names


def _init_store(store: ParamStore, cfg: EncoderConfig, generator: Optional[torch.Generator]):
    store.allocate("cpu", cfg.initializer_range, generator)
    for e in store.entries:
        if e.init == "linear_default":
            fan_in = e.shape[-1] if e.key.endswith(".weight") else store.by_key[e.key[:-4] + "weight"].shape[-1]
            bound = 1.0 / math.sqrt(fan_in)
            store.view(e.key, "master").uniform_(-bound, bound, generator=generator)
    # HF zeroes the padding row of word embeddings at init
    store.view("transformer.embeddings.word_embeddings.weight", "master")[cfg.pad_token_id].zero_()
    store.mark_master_dirty()


# ===================================================================================== autograd fns
class _Ctx:
    """Per-forward constants shared by the fused functions (not tensors)."""

    def __init__(self, B, L, seed, training, model):
        self.B, self.L, self.seed, self.training, self.model = B, L, seed, training, model
        self.x8 = {}   # fp8 path: layer index -> its QKV input in e4m3 (written by the previous layer's LN)
        self.head_mask = None   # [layers, H] per-column multipliers (each head's mask over its dh columns), or None
        # grad mode of the CALLER: inside an autograd.Function's forward torch.is_grad_enabled() is always False
        self.grad = torch.is_grad_enabled()


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, pos_ids, type_ids, info: _Ctx):
        m = info.model
        cfg = m.config
        st = m.store
        e = "transformer.embeddings."
        p = cfg.hidden_dropout_prob if info.training else 0.0
        y, mean, rstd = ops.embed_fwd(ids, pos_ids, type_ids, st.view(e + "word_embeddings.weight"),
                                      st.view(e + "position_embeddings.weight"),
                                      st.view(e + "token_type_embeddings.weight"),
                                      st.view(e + "LayerNorm.weight", "master"), st.view(e + "LayerNorm.bias", "master"),
                                      cfg.layer_norm_eps, p, info.seed, 0, st.compute_dtype)
        ctx.save_for_backward(ids, pos_ids, type_ids, mean, rstd)
        ctx.info, ctx.p = info, p
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, pos_ids, type_ids, mean, rstd = ctx.saved_tensors
        info = ctx.info
        m = info.model
        st = m.store
        e = "transformer.embeddings."
        acc = m._take_accumulate("embeddings")
        trainable = m.store.params[e + "word_embeddings.weight"].requires_grad
        if trainable:
            ops.embed_bwd(dy.contiguous(), ids, pos_ids, type_ids, st.view(e + "word_embeddings.weight"),
                          st.view(e + "position_embeddings.weight"), st.view(e + "token_type_embeddings.weight"),
                          st.view(e + "LayerNorm.weight", "master"), mean, rstd, ctx.p, info.seed, 0,
                          st.view(e + "word_embeddings.weight", "grad"), st.view(e + "position_embeddings.weight", "grad"),
                          st.view(e + "token_type_embeddings.weight", "grad"), st.view(e + "LayerNorm.weight", "grad"),
                          st.view(e + "LayerNorm.bias", "grad"), acc, m.config.pad_token_id,
                          m.config.pad_token_id if m.config.family == "roberta" else -1, info.L)
            m._group_ready("embeddings")
        return None, None, None, None, None


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, key_bias, idx: int, info: _Ctx):
        m = info.model
        cfg = m.config
        st = m.store
        B, L, nh = info.B, info.L, cfg.num_attention_heads
        p = f"transformer.encoder.layer.{idx}."
        ph = cfg.hidden_dropout_prob if info.training else 0.0
        pa = cfg.attention_probs_dropout_prob if info.training else 0.0
        scale = 1.0 / math.sqrt(cfg.head_dim)
        op0 = 1 + 3 * idx
        Bm = lambda k: st.view(p + k, "master")  # noqa: E731  (fp32 bias for the MFMA epilogue)
        fp8 = m.precision == "fp8" and x.is_cuda
        W8 = lambda k: st.view_fp8(p + k + ".weight")  # noqa: E731  (e4m3 weight + dequant scale)
        Bb = lambda k: st.view(p + k + ".bias")  # noqa: E731

        kinds = {"qkv": "qkv", "attention.output.dense": "out", "output.dense": "ffn2"}

        def proj(inp, name):  # bf16 forward projection
            return ops.linear_fwd(inp, st.view(p + name + ".weight"), Bb(name), Bm(name + ".bias"), kinds[name])

        # --precision fp8 (BASELINE config #5): every forward projection — QKV, out-projection, FFN1, FFN2
        # — runs on the own block-scaled fp8 MFMA kernel (gemm_fp8.hip) with e4m3 inputs written by their
        # PRODUCERS under delayed scaling: QKV's by the previous layer's second LayerNorm (layer 0: one
        # quantisation pass over the embeddings), the out-projection's by the attention forward's ctx store,
        # FFN1's by this layer's first LayerNorm, FFN2's by FFN1's epilogue — so no standalone quantiser
        # runs per layer.  In the backward every dgrad (FFN2, FFN1, out-projection, QKV) and the weight
        # gradients of the out-projection, FFN1 and FFN2 run in fp8 too (e5m2 gradients, see backward): the
        # e4m3 inputs written here are kept for those weight gradients.
        fp8 = fp8 and ops.fp8_gemm_ok(x.shape[0], 3 * cfg.hidden_size, cfg.hidden_size)
        s8 = m.fp8_states(idx) if fp8 else None
        # LayerNorm z only when the backward needs it (ops.LN_FROM_Y: recomputed from y on the GPU, for the
        # LayerNorms whose weights pass the |β| <= R·|γ| guard, BertForQuestionAnswering.refresh_ln_modes)
        keep_z = not (x.is_cuda and x.dtype != torch.float32 and ops.LN_FROM_Y)
        keep_z1 = keep_z or not m.ln_from_y_ok(idx, 0)
        keep_z2 = keep_z or not m.ln_from_y_ok(idx, 1)
        if fp8:
            x8 = info.x8.pop(idx, None)
            if x8 is None:
                x8 = s8["qkv"].quantize(x)
            qkv = ops.linear_fwd_fp8_own(x8, s8["qkv"], W8("qkv"), Bm("qkv.bias"))
        else:
            qkv = proj(x, "qkv")
        if fp8:
            ctxv, lse, bits, ctx8 = ops.attn_fwd_q8(qkv, key_bias, B, L, nh, pa, info.seed, op0, scale, s8["out"])
            a1 = ops.linear_fwd_fp8_own(ctx8, s8["out"], W8("attention.output.dense"),
                                        Bm("attention.output.dense.bias"))
        else:
            ctxv, lse, bits = ops.attn_fwd(qkv, key_bias, B, L, nh, pa, info.seed, op0, scale)
        # head_mask (HF: attention_probs *= head_mask[h]): scales head h's context, so the out-projection reads
        # ctx ⊙ mvec; ctxv (the unmasked attention output) stays what the attention backward recomputes against
        mvec = info.head_mask[idx] if info.head_mask is not None else None
        ctx_in = ctxv if mvec is None else (ctxv.float() * mvec).to(ctxv.dtype)
        ln1 = (st.view(p + "attention.output.LayerNorm.weight", "master"),
               st.view(p + "attention.output.LayerNorm.bias", "master"), cfg.layer_norm_eps, ph, info.seed, op0 + 1)
        h1_8 = None
        if fp8:
            h1, z1, m1, r1, h1_8 = ops.ln_fwd_q8(a1, x, *ln1, s8["ffn1"], store_z=keep_z1)
        else:   # out-projection + dropout + residual + LayerNorm (one GEMM epilogue + z-in LN under ops.LN_FUSE)
            name = "attention.output.dense"
            h1, z1, m1, r1 = ops.linear_bdr_ln_fwd(ctx_in, st.view(p + name + ".weight"), Bb(name), Bm(name + ".bias"),
                                                   x, kinds[name], *ln1, store_z=keep_z1)
        act8 = None
        # bf16 act is only read by a bf16 FFN2 weight gradient: skipped (604 MB of stores at b256) when the
        # backward will run that weight gradient in fp8 from act8 (its gradient state calibrated by then)
        need_act = not (fp8 and info.grad and m.fp8_backward_ok(x.shape[0])
                        and s8["dffn2"].step >= 1)
        r8 = (ops.linear_gelu_fwd_fp8(h1, W8("intermediate.dense"), Bm("intermediate.dense.bias"), s8["ffn1"],
                                      s8["ffn2"], x8=h1_8, need_act=need_act) if fp8 else None)
        if r8 is not None:
            pre, act, act8 = r8
            ctx.gelu_deriv = True
        else:  # `pre` holds gelu'(pre) when the fused MFMA epilogue ran (ctx.gelu_deriv)
            pre, act, ctx.gelu_deriv = ops.linear_gelu_fwd_d(h1, st.view(p + "intermediate.dense.weight"),
                                                             Bb("intermediate.dense"), Bm("intermediate.dense.bias"))
        ln2 = (st.view(p + "output.LayerNorm.weight", "master"), st.view(p + "output.LayerNorm.bias", "master"),
               cfg.layer_norm_eps, ph, info.seed, op0 + 2)
        if act8 is not None:
            a2 = ops.linear_fwd_fp8_own(act8, s8["ffn2"], W8("output.dense"), Bm("output.dense.bias"))
            if idx + 1 < cfg.num_hidden_layers:  # the next layer's QKV input, in e4m3
                h2, z2, m2, r2, info.x8[idx + 1] = ops.ln_fwd_q8(a2, h1, *ln2, m.fp8_states(idx + 1)["qkv"],
                                                                 store_z=keep_z2)
            else:
                h2, z2, m2, r2 = ops.ln_fwd(a2, h1, *ln2, store_z=keep_z2)
        else:   # FFN2 + dropout + residual + LayerNorm (one GEMM epilogue + z-in LN under ops.LN_FUSE)
            name = "output.dense"
            h2, z2, m2, r2 = ops.linear_bdr_ln_fwd(act, st.view(p + name + ".weight"), Bb(name), Bm(name + ".bias"), h1,
                                                   kinds[name], *ln2, store_z=keep_z2)
        # a LayerNorm without z (None) recomputes x̂ from its output y (h1 / h2) in the backward
        ctx.save_for_backward(x, key_bias, qkv, ctxv, lse, z1, m1, r1, h1, pre, act, z2, m2, r2,
                              h2 if z2 is None else None)
        # e4m3 inputs of the out-projection / FFN1 / FFN2 GEMMs (their scales stay in the states until the next
        # forward re-quantises), for the fp8 weight gradients
        ctx.f8 = (ctx8, h1_8, act8, x8) if (fp8 and act8 is not None and h1_8 is not None) else None
        ctx.bits = bits
        ctx.info, ctx.idx, ctx.ph, ctx.pa, ctx.scale = info, idx, ph, pa, scale
        ctx.mvec = mvec
        return h2

    @staticmethod
    def backward(ctx, dh2):
        x, key_bias, qkv, ctxv, lse, z1, m1, r1, h1, pre, act, z2, m2, r2, h2 = ctx.saved_tensors
        info = ctx.info
        m = info.model
        cfg = m.config
        st = m.store
        idx = ctx.idx
        B, L, nh = info.B, info.L, cfg.num_attention_heads
        p = f"transformer.encoder.layer.{idx}."
        op0 = 1 + 3 * idx
        grp = f"layer.{idx}"
        trainable = st.params[p + "attention.self.query.weight"].requires_grad
        acc = m._take_accumulate(grp) if trainable else False
        G = (lambda k: st.view(p + k, "grad")) if trainable else (lambda k: None)
        W = lambda k: st.view(p + k)  # noqa: E731
        WT = lambda k: st.view_t(p + k)  # noqa: E731  (Wᵀ working copy, GPU only)
        side = m.grad_side_stream if dh2.is_cuda else None

        def wgrad(dy, xin, gw, gb, q=None):  # dW (+db) — on the side stream when enabled (overlaps the dgrads)
            """q = (dy8, dy_state, x8, x_state): the fp8 form (no bias) once the gradient state is calibrated."""
            if not trainable:
                return
            use8 = (q is not None and q[0] is not None and q[2] is not None and q[1].calibrated
                    and ops.fp8_wgrad_ok(q[0].shape[0], q[0].shape[1], q[2].shape[1]))
            # the forward / DMUL skip a bf16 operand only when this fp8 form is certain to run
            assert use8 or (dy is not None and xin is not None), "bf16 weight-gradient operand was not kept"

            def run():
                if use8:
                    ops.linear_wgrad_fp8(q[0], q[1], q[2], q[3], gw, acc)
                else:
                    ops.linear_wgrad(dy, xin, gw, gb, acc)
            if side is None or use8:
                # fp8 runs on the compute stream: the kernel reads the delayed-scaling scale words (state buf[3])
                # when it executes, and the next micro-batch's forward producers rewrite them on this stream —
                # record_stream protects the operands' memory, not those values
                run()
                return
            side.wait_stream(torch.cuda.current_stream())
            for t in ((q[0], q[2]) if use8 else (dy, xin)):
                t.record_stream(side)
            with torch.cuda.stream(side):
                run()
        Wm = lambda k: st.view(p + k, "master")  # noqa: E731
        dh2 = dh2.contiguous()
        # --precision fp8: the FFN2 / FFN1 / out-projection / QKV dgrads run on the fp8 MFMA kernel with e5m2
        # gradients (range ±57344; e4m3's ±448 is too narrow for gradients) against the e4m3 Wᵀ copies —
        # each gradient written in e5m2 by its PRODUCER under delayed scaling: da2 and da1 by the LayerNorm
        # backwards, dpre by the FFN2 dgrad's DMUL epilogue, dQKV by the attention backward.  A gradient state has no current-scaling seed,
        # so its consumer runs in bf16 until one production has recorded an amax (``calibrated``).
        fp8 = m.precision == "fp8" and dh2.is_cuda and ctx.gelu_deriv and m.fp8_backward_ok(dh2.shape[0])
        s8 = m.fp8_states(idx) if fp8 else None
        W8T = lambda k: st.view_fp8_t(p + k)  # noqa: E731  (e4m3 Wᵀ + dequant scale)
        f8 = ctx.f8 if fp8 else None          # (ctx8, h1_8, act8, x8): e4m3 forward inputs for the fp8 wgrads
        ctx.f8 = None

        # --- FFN block ------------------------------------------------------------------------
        beta2 = Wm("output.LayerNorm.bias") if z2 is None else None   # x̂ from y (no stored z)
        ln2b = (dh2, None, z2 if z2 is not None else h2, Wm("output.LayerNorm.weight"), m2, r2, ctx.ph, info.seed,
                op0 + 2, G("output.LayerNorm.weight"), G("output.LayerNorm.bias"), G("output.dense.bias"), acc)
        if fp8:   # bf16 da2 only while its fp8 consumers (FFN2 dgrad + weight gradient) still fall back
            need = not (s8["dffn2"].step >= 1 and (f8 is not None or not trainable))
            dz2, da2, da2_8 = ops.ln_bwd_q8(*ln2b, s8["dffn2"], need, beta=beta2)
        else:
            dz2, da2 = ops.ln_bwd(*ln2b, beta=beta2)
        wgrad(da2, act, G("output.dense.weight"), None, (da2_8, s8["dffn2"], f8[2], s8["ffn2"]) if f8 else None)
        dpre8 = None
        if fp8 and s8["dffn2"].calibrated:
            # bf16 dpre only if a consumer still needs it: the FFN1 dgrad and weight gradient read dpre8 once
            # its state is calibrated (after this production), the latter only with the e4m3 h1 kept
            need_dpre = not (s8["dffn1"].step >= 1 and (f8 is not None or not trainable))
            dpre, dpre8 = ops.linear_dgrad_gelu_fp8(da2_8, s8["dffn2"], W8T("output.dense.weight"), pre,
                                                    G("intermediate.dense.bias"), acc, s8["dffn1"], need_dpre)
        else:
            dpre = ops.linear_dgrad_gelu_d(da2, W("output.dense.weight"), pre, ctx.gelu_deriv,
                                           G("intermediate.dense.bias"), acc, wt=WT("output.dense.weight"))
        wgrad(dpre, h1, G("intermediate.dense.weight"), None, (dpre8, s8["dffn1"], f8[1], s8["ffn1"]) if f8 else None)
        if dpre8 is not None and s8["dffn1"].calibrated:
            dh1_ffn = ops.linear_dgrad_fp8(dpre8, s8["dffn1"], W8T("intermediate.dense.weight"))
        else:
            dh1_ffn = ops.linear_dgrad(dpre, W("intermediate.dense.weight"), wt=WT("intermediate.dense.weight"))
        # --- attention block ------------------------------------------------------------------
        beta1 = Wm("attention.output.LayerNorm.bias") if z1 is None else None
        ln1b = (dz2, dh1_ffn, z1 if z1 is not None else h1, Wm("attention.output.LayerNorm.weight"), m1, r1, ctx.ph,
                info.seed, op0 + 1, G("attention.output.LayerNorm.weight"), G("attention.output.LayerNorm.bias"),
                G("attention.output.dense.bias"), acc)
        if fp8:   # likewise for the out-projection dgrad + weight gradient
            need = not (s8["dout"].step >= 1 and (f8 is not None or not trainable))
            dz1, da1, da1_8 = ops.ln_bwd_q8(*ln1b, s8["dout"], need, beta=beta1)
        else:
            dz1, da1 = ops.ln_bwd(*ln1b, beta=beta1)
        mvec = ctx.mvec
        ctx_in = ctxv if mvec is None else (ctxv.float() * mvec).to(ctxv.dtype)   # what the out-projection read
        wgrad(da1, ctx_in, G("attention.output.dense.weight"), None,
              (da1_8, s8["dout"], f8[0], s8["out"]) if f8 else None)
        if fp8 and s8["dout"].calibrated:
            dctx = ops.linear_dgrad_fp8(da1_8, s8["dout"], W8T("attention.output.dense.weight"))
        else:
            dctx = ops.linear_dgrad(da1, W("attention.output.dense.weight"), wt=WT("attention.output.dense.weight"))
        if mvec is not None:   # d(ctx ⊙ m)/d ctx: a masked head passes no gradient into its attention
            dctx = (dctx.float() * mvec).to(dctx.dtype)
        bpart = None
        if fp8:   # calibrated: e5m2 dQKV only (+ QKV bias-gradient partials), the fp8 QKV wgrad reads it with x8
            need = not (s8["dqkv"].step >= 1 and (f8 is not None or not trainable))
            dqkv, dqkv8, bpart = ops.attn_bwd_q8(dctx, qkv, ctxv, lse, key_bias, ctx.bits, B, L, nh, ctx.pa, ctx.scale,
                                                 s8["dqkv"], need)
        else:
            dqkv = ops.attn_bwd(dctx, qkv, ctxv, lse, key_bias, ctx.bits, B, L, nh, ctx.pa, info.seed, op0, ctx.scale)
        ctx.bits = None
        if bpart is not None:
            wgrad(None, None, G("qkv.weight"), None, (dqkv8, s8["dqkv"], f8[3], s8["qkv"]))
            if trainable:
                ops.colsum_into(bpart, G("qkv.bias"), acc)
        else:
            wgrad(dqkv, x, G("qkv.weight"), G("qkv.bias"))
        if trainable:
            m._group_ready(grp)
        if fp8 and s8["dqkv"].calibrated:
            dx = ops.linear_dgrad_add_fp8(dqkv8, s8["dqkv"], W8T("qkv.weight"), dz1)
        else:
            dx = ops.linear_dgrad_add(dqkv, W("qkv.weight"), dz1, wt=WT("qkv.weight"))
        return dx, None, None, None, None


class _SpanHeadFn(torch.autograd.Function):
    """position_outputs (Linear(H, 2) over the sequence, reference ``model.py:30,54-58``) as one HIP
    kernel each way: fp32 logits from the bf16 sequence; backward writes the bf16 sequence gradient
    (rank-2 outer product) and dW partials (deterministic), db = Σ g."""

    @staticmethod
    def forward(ctx, seq, w, b):
        from .._native import kernels
        B, L, H = seq.shape
        seq = seq.contiguous()
        ctx.save_for_backward(seq, w)
        return kernels().span_fwd(seq, w.detach().contiguous(), b.detach().contiguous()).view(B, L, 2)

    @staticmethod
    def backward(ctx, g):
        from .._native import kernels
        seq, w = ctx.saved_tensors
        g = g.float().contiguous()
        dw = torch.empty_like(w)
        dseq = kernels().span_bwd(seq, w.detach().contiguous(), g, dw, False)
        return dseq, dw, g.sum((0, 1))


# ============================================================================================ model
def _ensure_module(root: nn.Module, path: List[str]) -> nn.Module:
    mod = root
    for part in path:
        if not hasattr(mod, part) or not isinstance(getattr(mod, part), nn.Module):
            mod.add_module(part, nn.Module())
        mod = getattr(mod, part)
    return mod


class BertForQuestionAnswering(nn.Module):
    """Encoder + 5 QA outputs; ``forward(input_ids, attention_mask, token_type_ids, position_ids,
    head_mask) -> {start_class, end_class, start_reg, end_reg, cls}`` (reference ``model.py:43-73``)."""

    def __init__(self, config: EncoderConfig, *, device=None, precision: str = "bf16", seed: Optional[int] = None):
        super().__init__()
        self.config = config
        self.precision = precision
        self.fp8_dgrad = True   # --precision fp8: run the backward GEMMs (dgrads, most wgrads) in fp8 as well
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.store = ParamStore(build_entries(config))
        _init_store(self.store, config, gen)
        self.store.enable_transposed([f"transformer.encoder.layer.{i}.{k}" for i in range(config.num_hidden_layers)
                                      for k in ("qkv.weight", "attention.output.dense.weight",
                                                "intermediate.dense.weight", "output.dense.weight")])
        order = hf_param_order(config)
        assert sorted(order) == sorted(self.store.params), "param layout / HF order mismatch"
        for name in order:
            prm = self.store.params[name]
            *path, leaf = name.split(".")
            _ensure_module(self, path).register_parameter(leaf, prm)
        emb = _ensure_module(self, ["transformer", "embeddings"])
        emb.register_buffer("position_ids", torch.arange(config.max_position_embeddings).unsqueeze(0))
        # HQ_WGRAD_STREAM=1: weight-gradient GEMMs on a side stream, overlapping the dgrad/attention chain
        self.grad_side_stream = None
        self._want_side_stream = os.environ.get("HQ_WGRAD_STREAM", "0") == "1"
        self._head_params = [prm for n, prm in self.store.params.items() if not n.startswith("transformer.encoder")
                             and not n.startswith("transformer.embeddings")]
        self._fresh: Dict[str, bool] = {}
        self._grad_listener: Optional[Callable[[str], None]] = None
        self._head_pending = 0
        self._head_range = next((s, e) for g, s, e in self.store.group_ranges() if g == "head")
        for prm in self._head_params:
            prm.register_post_accumulate_grad_hook(self._head_hook)
        self.zero_grad()
        if device is not None:
            self.to(device)

    # -------------------------------------------------------------------- device / precision
    def __deepcopy__(self, memo):
        """Parameters are arena views, which ``copy.deepcopy`` would un-share: rebuild instead."""
        import copy as _copy
        new = type(self)(_copy.deepcopy(self.config), precision=self.precision)
        new.store.master.copy_(self.store.master.detach().cpu())
        new.store.mark_master_dirty()
        new.train(self.training)
        for n, p in self.named_parameters():
            dict(new.named_parameters())[n].requires_grad_(p.requires_grad)
        if self.store.device.type != "cpu":
            new.to(self.store.device)
        new.store.sync_compute()
        return new

    def _apply(self, fn, recurse=True):
        probe = fn(torch.empty(0, dtype=torch.float32, device=self.store.device))
        if probe.dtype != torch.float32:
            raise RuntimeError("Cast the compute precision with --precision; master weights stay fp32.")
        self.store.to(probe.device)
        self.store.set_compute_dtype(self.compute_dtype_for(probe.device))
        if probe.device.type == "cuda":
            if self._want_side_stream and self.grad_side_stream is None:
                self.grad_side_stream = torch.cuda.Stream(device=probe.device)
        else:
            self.grad_side_stream = None
        for mod in self.modules():
            for k, b in list(mod._buffers.items()):
                if b is not None:
                    mod._buffers[k] = fn(b)
        return self

    def use_device_seed(self, enable: bool):
        """Dropout kernels read their per-step seed from a device word (``seed_device``) instead of a
        launch argument — required inside a captured HIP graph, whose replays must draw new masks.  The
        registration is process-wide (one captured model per process)."""
        from .._native import kernels
        if enable:
            if getattr(self, "_seed_dev", None) is None or self._seed_dev.device != self.store.device:
                self._seed_dev = torch.zeros(1, dtype=torch.int32, device=self.store.device)
            kernels().set_dropout_seed(self._seed_dev)
        else:
            kernels().set_dropout_seed(None)

    @property
    def seed_device(self) -> Optional[torch.Tensor]:
        return getattr(self, "_seed_dev", None)

    def compute_dtype_for(self, device) -> torch.dtype:
        if torch.device(device).type != "cuda":
            return torch.float32
        return {"bf16": torch.bfloat16, "fp32": torch.float32, "fp8": torch.bfloat16}[self.precision]

    def fp8_backward_ok(self, T: int) -> bool:
        """The fp8 backward (e5m2 dgrads and weight gradients) runs for T tokens: enabled and every GEMM
        shape tiles on gemm_fp8 / gemm_tn8 (BERT / RoBERTa base and large at T % 256 == 0)."""
        c = self.config
        H, F = c.hidden_size, c.intermediate_size
        return (self.fp8_dgrad and ops.fp8_gemm_ok(T, F, H) and ops.fp8_gemm_ok(T, H, F) and ops.fp8_gemm_ok(T, H, H)
                and ops.fp8_gemm_ok(T, H, 3 * H) and ops.fp8_wgrad_ok(T, H, F) and ops.fp8_wgrad_ok(T, F, H)
                and ops.fp8_wgrad_ok(T, H, H) and ops.fp8_wgrad_ok(T, 3 * H, H))

    def fp8_states(self, idx: int):
        """Delayed-scaling states of layer ``idx``'s fp8 GEMM inputs (created on first use)."""
        if not hasattr(self, "_fp8_states"):
            self._fp8_states = {}
        st = self._fp8_states.get(idx)
        if st is None or st["qkv"].buf.device != self.store.device:
            st = {k: ops.Fp8DelayedState(self.store.device) for k in ("qkv", "out", "ffn1", "ffn2")}
            # activation gradients (e5m2): the inputs of the FFN2 / FFN1 / out-projection dgrads
            st.update({k: ops.Fp8DelayedState(self.store.device, grad=True)
                       for k in ("dffn2", "dffn1", "dout", "dqkv")})
            self._fp8_states[idx] = st
        return st

    def set_precision(self, precision: str):
        self.precision = precision
        self.store.set_compute_dtype(self.compute_dtype_for(self.store.device))

    @property
    def device(self):
        return self.store.device

    # -------------------------------------------------------------------- grads / reducer hooks
    def zero_grad(self, set_to_none: bool = False):
        """Mark every gradient group "fresh": the next backward overwrites instead of accumulating (no
        memset of the arena).  The autograd heads path clears the head range lazily in ``forward``."""
        for g, s, e in self.store.group_ranges():
            self._fresh[g] = True
        self._head_pending = len([p for p in self._head_params if p.requires_grad])

    def _take_accumulate(self, group: str) -> bool:
        fresh = self._fresh.get(group, True)
        self._fresh[group] = False
        return not fresh

    def _group_ready(self, group: str):
        if self._grad_listener is not None:
            self._grad_listener(group)

    def _head_hook(self, _p):
        self._head_pending -= 1
        if self._head_pending == 0:
            self._group_ready("head")
            self._head_pending = len([p for p in self._head_params if p.requires_grad])

    def set_grad_listener(self, fn: Optional[Callable[[str], None]]):
        self._grad_listener = fn

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        state_dict = dict(state_dict)
        pid = "transformer.embeddings.position_ids"
        if pid not in state_dict:
            state_dict[pid] = self.transformer.embeddings.position_ids.clone()
        res = super().load_state_dict(state_dict, strict=strict)
        self.store.mark_master_dirty()
        self.store.sync_compute()
        # new LayerNorm weights: re-run the from-y guard NOW (outside any graph capture — its one device→host
        # read must never land inside a capture of the next forward) and bump the mode version, which makes a
        # TrainEngine with live graphs re-capture them
        self._ln_y = None
        self._ln_pending = None
        self.refresh_ln_modes()
        self.ln_mode_version = getattr(self, "ln_mode_version", 0) + 1
        return res

    # -------------------------------------------------------------------- LayerNorm-from-y guard
    # The memory-efficient LayerNorm backward recomputes x̂ = (y − β)/γ from the bf16 output y; y's rounding
    # (2⁻⁹·|y|, |y| <= |γ|·|x̂| + |β|) puts 2⁻⁹·(|x̂| + |β/γ|) into x̂ — the same class as the stored-z form's
    # 2⁻⁹·|z|·rstd while |β/γ| stays O(|x̂|), but unbounded for a small-|γ| column (γ = 0: x̂ is lost).
    # Random-init weights (γ = 1, β = 0) always pass; pretrained checkpoints are checked column by column.
    LN_FROM_Y_MAX_RATIO = 8.0

    def _ln_names(self):
        return [f"transformer.encoder.layer.{i}.{k}" for i in range(self.config.num_hidden_layers)
                for k in ("attention.output.LayerNorm", "output.LayerNorm")]

    def refresh_ln_modes(self) -> bool:
        """Re-evaluate, per encoder LayerNorm, whether the from-y backward is safe: every column has γ != 0 and
        |β| <= LN_FROM_Y_MAX_RATIO·|γ|; a LayerNorm that fails stores z instead.  One small device→host read.
        Returns True when a LayerNorm changed mode (a captured HIP graph must then be re-captured)."""
        return self._apply_ln_flags(self._ln_flags().tolist())

    def _ln_flags(self) -> torch.Tensor:
        names = self._ln_names()
        m = self.store.master
        if m.is_cuda:   # one own kernel (norm.hip ln_guard_kernel) over the master arena, no ATen chain
            offs = getattr(self, "_ln_guard_offs", None)
            if offs is None or offs[0].device != m.device:
                H = self.config.hidden_size
                def off(n):
                    v = self.store.view(n, "master")
                    o = (v.data_ptr() - m.data_ptr()) // m.element_size()
                    assert v.is_contiguous() and v.numel() == H and 0 <= o and o + H <= m.numel(), n
                    return o
                offs = self._ln_guard_offs = (
                    torch.tensor([off(n + ".weight") for n in names], dtype=torch.int64, device=m.device),
                    torch.tensor([off(n + ".bias") for n in names], dtype=torch.int64, device=m.device))
            from .._native import kernels
            return kernels().ln_guard(m, offs[0], offs[1], self.config.hidden_size, self.LN_FROM_Y_MAX_RATIO)
        g = torch.stack([self.store.view(n + ".weight", "master") for n in names]).abs()
        b = torch.stack([self.store.view(n + ".bias", "master") for n in names]).abs()
        return ((g > 0) & (b <= self.LN_FROM_Y_MAX_RATIO * g)).all(1)

    def _apply_ln_flags(self, ok) -> bool:
        old = getattr(self, "_ln_y", None)
        self._ln_y = [bool(v) for v in ok]
        changed = old is not None and old != self._ln_y
        if changed:
            self.ln_mode_version = getattr(self, "ln_mode_version", 0) + 1
        return changed

    def poll_ln_modes(self) -> bool:
        """Asynchronous form of ``refresh_ln_modes`` for the training loop: applies the flags of the check launched
        at the previous call, then launches the next check (a few tiny kernels + a non-blocking copy into pinned
        memory behind an event) on the current stream.  The previous check was launched ``ln_check_every`` optimizer
        steps ago, so waiting for its event costs nothing in practice — and waiting (rather than polling) makes
        every data-parallel rank apply a mode change at the SAME optimizer step, so replicas stay bitwise
        reproducible and release / recapture their graphs together.  Returns True when a LayerNorm changed mode."""
        changed = False
        pend = getattr(self, "_ln_pending", None)
        if pend is not None:
            host, ev = pend
            ev.synchronize()
            changed = self._apply_ln_flags(host.tolist())
        flags = self._ln_flags()
        host = torch.empty(flags.shape, dtype=torch.bool, pin_memory=True)
        host.copy_(flags, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ln_pending = (host, ev)
        return changed

    def ln_from_y_ok(self, idx: int, which: int) -> bool:
        """Layer ``idx``'s LayerNorm ``which`` (0 = attention output, 1 = FFN output) may skip storing z."""
        if getattr(self, "_ln_y", None) is None:
            self.refresh_ln_modes()
        return self._ln_y[2 * idx + which]

    # -------------------------------------------------------------------- forward
    def _position_ids(self, input_ids, position_ids):
        B, L = input_ids.shape
        if position_ids is not None:
            return position_ids.expand(B, L)
        if self.config.family == "roberta":
            mask = input_ids.ne(self.config.pad_token_id).to(torch.int64)
            return torch.cumsum(mask, dim=1) * mask + self.config.pad_token_id
        return self.transformer.embeddings.position_ids[:, :L].expand(B, L)

    def _default_positions(self, B: int, L: int, dev) -> torch.Tensor:
        """BERT's default position ids (0 … L-1 for every row) flattened to [B·L] int64, cached per shape: the
        forward used to expand + copy them every step."""
        cache = self.__dict__.setdefault("_pos_cache", {})
        # entries read inside a HIP-graph capture stay pinned: the captured kernels keep their address, so the
        # tensor must outlive the graph (a cleared entry's memory would be handed to later allocations)
        pinned = self.__dict__.setdefault("_pos_pinned", set())
        key = (B, L, str(dev))
        t = cache.get(key)
        if t is None:
            if len(cache) >= 8:
                for k in [k for k in cache if k not in pinned]:
                    del cache[k]
            t = cache[key] = self.transformer.embeddings.position_ids[0, :L].to(dev, torch.int64).repeat(B).contiguous()
        if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            pinned.add(key)
        return t

    def encode(self, input_ids, attention_mask=None, token_type_ids=None, position_ids=None):
        return self._encode(input_ids, attention_mask, token_type_ids, position_ids)[0]

    def _head_mask_columns(self, head_mask):
        """HF ``get_head_mask`` shapes — [nh] (every layer) or [layers, nh] — as per-layer column multipliers
        [layers, H] (head h covers columns h·dh … h·dh+dh-1 of the attention context); None when all ones."""
        cfg = self.config
        nh, NL = cfg.num_attention_heads, cfg.num_hidden_layers
        hm = torch.as_tensor(head_mask, dtype=torch.float32, device=self.store.device)
        if hm.dim() == 1:
            hm = hm.unsqueeze(0).expand(NL, nh)
        hm = hm.reshape(NL, nh) if hm.numel() == NL * nh else None
        if hm is None:
            raise ValueError(f"head_mask must have {nh} or {NL}x{nh} elements, got shape {tuple(head_mask.shape)}")
        if bool((hm == 1).all()):
            return None
        if self.precision == "fp8" and self.store.device.type == "cuda":
            raise NotImplementedError("head_mask with --precision fp8 (the fp8 out-projection reads the attention "
                                      "kernel's e4m3 context directly)")
        return hm.repeat_interleave(cfg.head_dim, dim=1).contiguous()

    def _encode(self, input_ids, attention_mask=None, token_type_ids=None, position_ids=None, head_mask=None):
        cfg = self.config
        B, L = input_ids.shape
        if L > cfg.max_position_embeddings - cfg.position_offset:
            raise ValueError(f"sequence length {L} exceeds max positions {cfg.max_position_embeddings}")
        self.store.sync_compute()
        dev = self.store.device
        ids = input_ids.reshape(-1).to(dev, torch.int64)
        tt = (token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)).reshape(-1).to(dev, torch.int64)
        if position_ids is None and self.config.family != "roberta" and dev.type == "cuda":
            pos = self._default_positions(B, L, dev)   # cached [B·L] arange rows: no per-step expand copy
        else:
            pos = self._position_ids(input_ids, position_ids).reshape(-1).to(dev, torch.int64)
        if attention_mask is None:
            key_bias = torch.zeros(B, L, dtype=torch.float32, device=dev)
        elif dev.type == "cuda" and attention_mask.dtype in (torch.bool, torch.uint8):
            from .._native import kernels   # one own kernel (norm.hip key_bias_kernel)
            key_bias = kernels().key_bias(attention_mask.to(dev).contiguous())
        else:
            key_bias = (1.0 - attention_mask.to(dev, torch.float32)) * -10000.0
        # per-module train/eval as the reference's finetune mode sets it (model.eval() + .train() on the trainable
        # modules, trainer.py:227-234): the encoder's dropout follows `transformer`, the classifier's `classifier`
        enc_train = self.transformer.training
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if (enc_train or self.classifier.training) else 0
        info = _Ctx(B, L, seed, enc_train, self)
        if head_mask is not None:
            info.head_mask = self._head_mask_columns(head_mask)
        anchor_e = self.store.params["transformer.embeddings.word_embeddings.weight"]
        h = _EmbeddingFn.apply(anchor_e, ids, pos, tt, info)
        for i in range(cfg.num_hidden_layers):
            anchor = self.store.params[f"transformer.encoder.layer.{i}.attention.self.query.weight"]
            h = _LayerFn.apply(h, anchor, key_bias, i, info)
        return h.view(B, L, cfg.hidden_size), seed

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, position_ids=None, head_mask=None):
        """``head_mask`` (reference ``model.py:43-48`` → HF BertModel): [nh] or [layers, nh] multipliers of each
        head's attention probabilities; a zero head contributes nothing and receives no gradient."""
        seq, seed = self._encode(input_ids, attention_mask, token_type_ids, position_ids, head_mask)
        if fused_heads_available(self, seq):
            return fused_heads(self, seq, seed, self.classifier.training)
        if torch.is_grad_enabled() and self._fresh.get("head", True):
            # autograd accumulates into the arena views: clear the head range once per fresh step
            s, e = self._head_range
            self.store.grad[s:e].zero_()
            self._fresh["head"] = False
        span = _SpanHeadFn.apply if seq.is_cuda and seq.dtype == torch.bfloat16 else None
        return reference_heads(self, seq, seed, self.classifier.training, span_fn=span)


def load_pretrained(model: BertForQuestionAnswering, path: str) -> List[str]:
    """Load HF-named encoder weights from a local file/dir (safetensors or weights-only torch pickle).
    Keys may be bare (``embeddings.…``), ``bert.``/``roberta.``-prefixed or already ``transformer.``-prefixed."""
    import os
    files = []
    if os.path.isdir(path):
        for fn in ("model.safetensors", "pytorch_model.bin"):
            if os.path.exists(os.path.join(path, fn)):
                files.append(os.path.join(path, fn))
                break
    else:
        files.append(path)
    if not files:
        raise FileNotFoundError(f"no weights in {path}")
    f = files[0]
    if f.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(f)
    else:
        sd = torch.load(f, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
            sd = sd["model"]
    own = model.state_dict()
    mapped = {}
    for k, v in sd.items():
        k2 = k
        for pre in ("bert.", "roberta."):
            if k2.startswith(pre):
                k2 = k2[len(pre):]
        k2 = k2.replace("LayerNorm.gamma", "LayerNorm.weight").replace("LayerNorm.beta", "LayerNorm.bias")
        if not k2.startswith("transformer.") and ("transformer." + k2) in own:
            k2 = "transformer." + k2
        if k2 in own and own[k2].shape == v.shape:
            mapped[k2] = v
    missing = [k for k in own if k not in mapped]
    model.load_state_dict({**own, **mapped}, strict=True)
    return missing
