"""QA heads (pooler + position_outputs + classifier + reg_start/reg_end) and the fused loss path.

Reference: ``modules/model/model/model.py:27-41,54-73`` (heads), ``modules/model/model/loss.py:5-106`` and
``modules/init.py:18-40`` (losses).  Two implementations with identical semantics:

* ``reference_heads`` — plain fp32 PyTorch autograd on the master weights (CPU, fp32 precision, and the
  numerics oracle of the tests).  Autograd accumulates into the arena gradient views.
* the fused GPU path — ``csrc/kernels/heads.hip``: ONE launch for the pooler, the span logits and the
  small heads (``_FusedHeadsFn``), ONE for all five losses and their gradients w.r.t. the predictions
  (``fused_loss``, called by ``WeightedLoss``), ONE for the whole heads backward (+ the span weight
  column-sum), writing the head gradients straight into the arena and signalling the reducer's "head"
  bucket — instead of ~70 small ATen launches per micro-batch.

The loss kernel computes d(total)/d(preds) in its forward; its autograd backward only hands those
buffers (and the incoming scalar, e.g. ``1/batch_split``) to the heads backward, which recognises them
by address and scales inside the kernel.  Any other gradient (e.g. a custom loss over the same
predictions) takes the general path: the incoming gradients are packed and used as they are.

The classifier dropout uses the framework's counter-hash RNG (``ops.rng``, stream ``HEAD_DROPOUT_OPID``)
in both implementations, so the fused and reference paths draw the same mask.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import rng

HEAD_DROPOUT_OPID = 0x7FFF0001
_HS = 16  # row stride of the per-sample head-gradient buffer (class logits, then 8 / 9 = reg start / end)

_W_KEYS = ["transformer.pooler.dense.weight", "transformer.pooler.dense.bias", "classifier.1.weight",
           "classifier.1.bias", "reg_start.0.weight", "reg_start.0.bias", "reg_end.0.weight", "reg_end.0.bias",
           "position_outputs.weight", "position_outputs.bias"]


class HeadOutputs(dict):
    """The model's prediction dict; ``fused`` is the kernel state when the fused heads produced it."""
    fused: Optional["_FusedState"] = None


class _FusedState:
    def __init__(self, model, B, L, NL, seed, p, logits, pooled, cls, reg):
        self.model, self.B, self.L, self.NL, self.seed, self.p = model, B, L, NL, seed, p
        self.logits, self.pooled, self.cls, self.reg = logits, pooled, cls, reg
        self.outputs = None          # the five prediction tensors, to recognise them in the loss
        self.dlog = self.dheads = self.gscale = self.losses = None

    def owns(self, preds) -> bool:
        return self.outputs is not None and all(preds.get(k) is t for k, t in self.outputs.items())

    def grads_from_loss(self, d_s, d_e, d_rs, d_re, d_cls) -> bool:
        """True iff the incoming gradients are exactly the fused loss's buffers (unmodified)."""
        if self.gscale is None or self.dlog is None:
            return False
        lp, hp = self.dlog.data_ptr(), self.dheads.data_ptr()
        want = ((d_s, lp, (2 * self.L, 2)), (d_e, lp + 4, (2 * self.L, 2)), (d_rs, hp + 32, (_HS,)),
                (d_re, hp + 36, (_HS,)), (d_cls, hp, (_HS, 1)))
        return all(t is not None and t.data_ptr() == ptr and t.stride() == st for t, ptr, st in want)


def head_views(store, which: str) -> List[torch.Tensor]:
    return [store.view(k, which) for k in _W_KEYS]


def fused_heads_possible(model) -> bool:
    """The model's forward will take the fused head kernels on a bf16 / fp32 GPU sequence (config / flags only).
    Frozen head parameters (``--finetune_*``, reference D16) are fine: the backward kernel's gradients for them
    are cleared again, so they never reach the grad norm, the reducer or the optimizer."""
    cfg = model.config
    if os.environ.get("HQ_FUSED_HEADS", "1") == "0":
        return False
    return not (cfg.hidden_size % 64 or cfg.hidden_size > 2048 or not 1 <= cfg.num_labels <= 8)


def fused_heads_available(model, seq: torch.Tensor) -> bool:
    """bf16 (bf16 / fp8 step) or fp32 (--precision fp32) GPU sequences: heads.hip widens either to fp32."""
    return seq.is_cuda and seq.dtype in (torch.bfloat16, torch.float32) and fused_heads_possible(model)


class _FusedHeadsFn(torch.autograd.Function):
    """Autograd node over the (already computed) fused-head outputs; backward = one kernel + colsum."""

    @staticmethod
    def forward(ctx, seq, anchor, st: "_FusedState"):
        ctx.st = st
        ctx.save_for_backward(seq)
        lg = st.logits.view(st.B, st.L, 2)
        return lg[..., 0], lg[..., 1], st.reg[:, 0], st.reg[:, 1], st.cls

    @staticmethod
    def backward(ctx, d_s, d_e, d_rs, d_re, d_cls):
        from .._native import kernels
        (seq,) = ctx.saved_tensors
        st = ctx.st
        B, L, NL = st.B, st.L, st.NL
        if st.grads_from_loss(d_s, d_e, d_rs, d_re, d_cls):
            dlog, dheads, gscale = st.dlog, st.dheads, st.gscale
        else:  # general path: pack whatever arrived (None = that output did not reach the loss)
            dev = seq.device
            z = torch.zeros(B, L, device=dev)
            dlog = torch.stack([(d_s if d_s is not None else z).float(), (d_e if d_e is not None else z).float()],
                               -1).contiguous()
            dheads = torch.zeros(B, _HS, device=dev)
            if d_cls is not None:
                dheads[:, :NL] = d_cls.float()
            if d_rs is not None:
                dheads[:, 8] = d_rs.float()
            if d_re is not None:
                dheads[:, 9] = d_re.float()
            if st.gscale is not None and st.dlog is not None:
                # the fused loss handed its UNSCALED d(loss)/d(preds) buffers to autograd (the fast path scales
                # them in the kernel); here autograd has summed them with other gradients, so add the missing
                # (g - 1)·buffer to get g·fused + other
                c = st.gscale - 1.0
                dlog = dlog + c * st.dlog
                dheads[:, :NL] += c * st.dheads[:, :NL]
                dheads[:, 8:10] += c * st.dheads[:, 8:10]
            gscale = None
        st.gscale = None
        m = st.model
        acc = m._take_accumulate("head")
        dseq = kernels().qa_heads_bwd(seq, L, dlog.view(-1, 2), dheads, gscale, st.pooled, st.reg,
                                      head_views(m.store, "master"), head_views(m.store, "grad"), acc, st.p, st.seed,
                                      HEAD_DROPOUT_OPID)
        for k in _W_KEYS:   # frozen heads (finetune modes): no gradient, as autograd would leave them
            if not m.store.params[k].requires_grad:
                m.store.view(k, "grad").zero_()
        m._group_ready("head")
        return dseq, None, None


def fused_heads(model, seq: torch.Tensor, seed: int, training: bool) -> HeadOutputs:
    from .._native import kernels
    B, L, _ = seq.shape
    p = model.config.hidden_dropout_prob if training else 0.0
    seq = seq.contiguous()
    logits, pooled, cls, reg = kernels().qa_heads_fwd(seq, L, head_views(model.store, "master"), p, seed,
                                                      HEAD_DROPOUT_OPID)
    st = _FusedState(model, B, L, model.config.num_labels, seed, p, logits, pooled, cls, reg)
    P = model.store.params
    anchor = next((P[k] for k in _W_KEYS if P[k].requires_grad), P[_W_KEYS[0]])   # any trainable head parameter
    if torch.is_grad_enabled() and (seq.requires_grad or anchor.requires_grad):
        s, e, rs, re_, c = _FusedHeadsFn.apply(seq, anchor, st)
    else:
        lg = logits.view(B, L, 2)
        s, e, rs, re_, c = lg[..., 0], lg[..., 1], reg[:, 0], reg[:, 1], cls
    out = HeadOutputs(start_class=s, end_class=e, start_reg=rs, end_reg=re_, cls=c)
    out.fused = st
    st.outputs = dict(out)
    return out


def reference_heads(model, seq: torch.Tensor, seed: int, training: bool, span_fn=None) -> HeadOutputs:
    """fp32 autograd heads on the master weights (the numerics oracle of the fused kernels).  ``span_fn``
    optionally replaces the position_outputs Linear (the bf16-input span kernel of the unfused GPU path)."""
    P = model.store.params
    pooled = torch.tanh(F.linear(seq[:, 0].float(), P["transformer.pooler.dense.weight"],
                                 P["transformer.pooler.dense.bias"]))
    if span_fn is not None:
        pos_logits = span_fn(seq, P["position_outputs.weight"], P["position_outputs.bias"])
    else:
        pos_logits = F.linear(seq.float(), P["position_outputs.weight"], P["position_outputs.bias"])
    start_logits, end_logits = pos_logits.split(1, dim=-1)
    p = model.config.hidden_dropout_prob if training else 0.0
    cls_in = rng.dropout_apply(pooled, seed, HEAD_DROPOUT_OPID, p) if p > 0 else pooled
    cls = F.linear(cls_in, P["classifier.1.weight"], P["classifier.1.bias"])
    reg_start = torch.sigmoid(F.linear(pooled, P["reg_start.0.weight"], P["reg_start.0.bias"])).squeeze(-1)
    reg_end = torch.sigmoid(F.linear(pooled, P["reg_end.0.weight"], P["reg_end.0.bias"])).squeeze(-1)
    return HeadOutputs(start_class=start_logits.squeeze(-1), end_class=end_logits.squeeze(-1), start_reg=reg_start,
                       end_reg=reg_end, cls=cls)


# ================================================================================== fused loss
class FusedLossConfig:
    """Kernel parameters of a ``WeightedLoss`` whose five terms the loss kernel implements exactly."""

    def __init__(self, kind: int, ignore_cls: int, weights: List[float], alpha=1.0, gamma=2.0, conf=1.0, fill=0.0,
                 label_weights: Optional[torch.Tensor] = None, n_classes: Optional[int] = None):
        self.kind, self.ignore_cls, self.weights = kind, ignore_cls, [float(w) for w in weights]
        self.alpha, self.gamma, self.conf, self.fill = float(alpha), float(gamma), float(conf), float(fill)
        self.label_weights = label_weights
        self.n_classes = n_classes
        self._lw_dev: Dict[torch.device, torch.Tensor] = {}

    def lw(self, device):
        if self.label_weights is None:
            return None
        t = self._lw_dev.get(device)
        if t is None:
            t = self._lw_dev[device] = self.label_weights.detach().float().contiguous().to(device)
        return t


def fused_loss_config(losses: Dict[str, tuple]) -> Optional[FusedLossConfig]:
    """Map the reference loss modules onto the kernel's closed set; None = use the module path."""
    from .losses import FocalLossWithLogits, LabelSmoothingLossWithLogits
    keys = ["start_class", "end_class", "start_reg", "end_reg", "cls"]
    if sorted(losses) != sorted(keys):
        return None
    weights = [losses[k][1] for k in keys]
    if not all(isinstance(w, (int, float)) for w in weights):
        return None

    def plain_ce(m, ignore):
        return (type(m) is nn.CrossEntropyLoss and m.weight is None and m.ignore_index == ignore
                and m.reduction == "mean" and m.label_smoothing == 0.0)
    if not (plain_ce(losses["start_class"][0], -1) and plain_ce(losses["end_class"][0], -1)):
        return None
    for k in ("start_reg", "end_reg"):
        m = losses[k][0]
        if not (type(m) is nn.MSELoss and m.reduction == "mean"):
            return None
    c = losses["cls"][0]
    if type(c) is nn.CrossEntropyLoss:
        if c.reduction != "mean" or c.label_smoothing != 0.0:
            return None
        return FusedLossConfig(0, c.ignore_index, weights, label_weights=c.weight)
    if type(c) is FocalLossWithLogits:
        if c.reduction != "mean" or c.ignore_index != -1:
            return None
        return FusedLossConfig(1, -1, weights, alpha=c.alpha, gamma=c.gamma)
    if type(c) is LabelSmoothingLossWithLogits:
        if c.smoothing <= 0.0:
            return FusedLossConfig(0, c.ignore_index, weights, n_classes=c.n_classes)
        if 0 <= c.ignore_index < c.n_classes:
            return None
        fill = c.smoothing / (c.n_classes - c.num_ignore_ixs)
        return FusedLossConfig(2, c.ignore_index, weights, conf=c.confidence, fill=fill, n_classes=c.n_classes)
    return None


class _FusedLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, e, rs, re_, cls, st: _FusedState, cfg: FusedLossConfig, t_start, t_end, t_rs, t_re, t_cls,
                seg=None):
        from .._native import kernels
        losses, dlog, dheads = kernels().qa_loss(st.logits, st.cls, st.reg, t_start, t_end, t_rs, t_re, t_cls,
                                                 cfg.lw(st.logits.device), cfg.kind, cfg.ignore_cls, cfg.weights,
                                                 cfg.alpha, cfg.gamma, cfg.conf, cfg.fill, seg)
        st.dlog, st.dheads, st.losses = dlog.view(st.B, st.L, 2), dheads, losses
        ctx.st = st
        return losses[5]

    @staticmethod
    def backward(ctx, g):
        st = ctx.st
        st.gscale = g.detach().float().reshape(1).contiguous()
        dl, dh = st.dlog, st.dheads
        return (dl[..., 0], dl[..., 1], dh[:, 8], dh[:, 9], dh[:, :st.NL], None, None, None, None, None, None, None,
                None)


def fused_loss(preds: HeadOutputs, targets, cfg: FusedLossConfig):
    """(total loss, per-term device losses [6]) with the prediction gradients precomputed.  ``targets
    ["segments"]`` (int32 [S], optional): the batch is S merged micro-batches with those span lengths — every
    term is normalised per segment and averaged over them (``data.collate.merge_micro_batches``)."""
    st = preds.fused
    dev = st.logits.device

    def t(k, dt):
        return targets[k].to(dev, dt, non_blocking=True).reshape(-1).contiguous()
    seg = targets.get("segments")
    if seg is not None:
        seg = seg.to(dev, torch.int32, non_blocking=True).contiguous()
    total = _FusedLossFn.apply(preds["start_class"], preds["end_class"], preds["start_reg"], preds["end_reg"],
                               preds["cls"], st, cfg, t("start_class", torch.int64), t("end_class", torch.int64),
                               t("start_reg", torch.float32), t("end_reg", torch.float32), t("cls", torch.int64), seg)
    return total, st.losses


def fused_loss_usable(preds, cfg: Optional[FusedLossConfig]) -> bool:
    st = getattr(preds, "fused", None)
    if cfg is None or st is None or not st.owns(preds):
        return False
    return cfg.n_classes is None or cfg.n_classes == st.NL
