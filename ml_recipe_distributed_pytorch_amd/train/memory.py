"""HBM memory model of one training step and the per-GPU batch sizing it drives (SURVEY §7.6 item 8,
BASELINE config #4 "288 GB HBM per-GPU batch sizing").

The reference split ``train_batch_size`` into ``batch_split`` micro-batches by hand (``config/test_bert.cfg``:
256 = 128 × 2, sized for a 12 GB K80).  On a 288 GB MI355X the same global batch usually fits in ONE
micro-batch; ``plan_batch_split`` picks the smallest split whose micro-batch fits, from an analytic model
of what the fused encoder keeps alive (``models/bert.py::_LayerFn.forward`` ``save_for_backward`` list):

per layer and sample (L tokens, bf16 = 2 B):
    x, qkv (3H), ctx, z1, h1, z2 ........... 2·L·(8H)        (the layer input x is the previous h2)
    gelu'(pre), act (F each) ............... 2·L·(2F)
    LSE (nh f32), 4 LN row statistics ...... 4·L·(nh + 4)
    attention dropout keep-bits ............ nh·L²/8
plus the backward's transient working set of one layer (dpre, dqkv, ~6 [L, H] gradients, split-K slabs),
the embedding / heads activations and the parameter state (fp32 master + bf16 compute copy + bf16 Wᵀ
copies of the encoder weights + fp32 grad + AdamW m, v = 22 B per parameter).

``tests/test_memory_model.py`` pins the formula on CPU; ``tests/test_model_gpu.py`` checks it against
``torch.cuda.max_memory_allocated`` of real steps (within 15 %).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

BYTES_PER_PARAM = 4 + 2 + 4 + 8          # fp32 master, bf16 compute copy, fp32 grad, AdamW m + v
BYTES_PER_ENCODER_WEIGHT_T = 2           # bf16 Wᵀ working copy for the dgrad GEMMs (encoder matrices only)


@dataclass
class MemoryEstimate:
    params_bytes: int
    act_bytes_per_sample: int
    transient_bytes_per_sample: int

    def total(self, micro_batch: int) -> int:
        return self.params_bytes + micro_batch * (self.act_bytes_per_sample + self.transient_bytes_per_sample)


def estimate(cfg, seq_len: int) -> MemoryEstimate:
    """Analytic HBM use of one optimizer step of ``BertForQuestionAnswering`` built from ``cfg``."""
    H, F, nh, NL, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.num_hidden_layers, seq_len
    n_enc_w = NL * (4 * H * H + 2 * H * F)                                     # QKV, out, FFN1, FFN2 matrices
    n_params = (cfg.vocab_size + cfg.max_position_embeddings + cfg.type_vocab_size + 2) * H \
        + NL * (4 * H * H + 2 * H * F + 9 * H + F) + H * H + H + 8 * (H + 1)  # + pooler + QA heads
    params = n_params * BYTES_PER_PARAM + n_enc_w * BYTES_PER_ENCODER_WEIGHT_T
    per_layer = 2 * L * (8 * H + 2 * F) + 4 * L * (nh + 4) + nh * L * L // 8
    emb_heads = 2 * L * H * 2 + 4 * L * 4 + 8 * L * 4                            # embedding out, LN stats, logits
    act = NL * per_layer + emb_heads
    # one layer's backward in flight: dpre [L,F] + dqkv [L,3H] + ~6 [L,H] gradients (bf16) + the attention
    # backward's δ (nh f32); the forward's own temporaries (a1, a2 before LayerNorm) are smaller
    transient = 2 * L * (F + 3 * H + 6 * H) + 4 * L * nh
    return MemoryEstimate(params, act, transient)


def max_micro_batch(cfg, seq_len: int, hbm_bytes: float, headroom: float = 0.9) -> int:
    """Largest micro-batch whose modelled step fits in ``headroom`` × ``hbm_bytes``."""
    est = estimate(cfg, seq_len)
    budget = headroom * hbm_bytes - est.params_bytes
    per = est.act_bytes_per_sample + est.transient_bytes_per_sample
    return max(0, int(budget // per))


def plan_batch_split(cfg, seq_len: int, train_batch_size: int, hbm_bytes: float, requested: int = 1,
                     headroom: float = 0.9, merge: bool = True) -> int:
    """Smallest accumulation split that divides ``train_batch_size`` and whose micro-batch fits the memory
    model (the reference's ``--batch_split`` semantics: micro = train_batch_size // split).  ``merge=True``
    may go BELOW ``requested`` (the reference config's 128 micro-batches of 2, sized for a 12 GB K80,
    become one micro-batch of 256 on a 288 GB MI355X); ``merge=False`` only ever raises it."""
    cap = max_micro_batch(cfg, seq_len, hbm_bytes, headroom)
    lo = 1 if merge else max(1, requested)
    for split in range(lo, train_batch_size + 1):
        if train_batch_size % split == 0 and train_batch_size // split <= max(cap, 1):
            return split
    return train_batch_size


def plan_exact_merge(cfg, seq_len: int, train_batch_size: int, hbm_bytes: float, requested: int = 1,
                     headroom: float = 0.9):
    """(batch_split, merge_segments) for the exact-objective merge (the GPU default of --auto_batch_split).

    The DataLoader keeps the reference's micro-batches (``requested`` of them, each collated on its own); the
    engine runs them in as few merged passes P as fit the memory model, P dividing ``requested``, each pass
    holding ``merge_segments`` = requested / P micro-batches as loss segments — the reference objective at
    merged-batch speed.  When even one micro-batch does not fit, the split is raised as ``plan_batch_split``
    (merge=False) does and nothing is merged."""
    requested = max(1, int(requested))
    cap = max(max_micro_batch(cfg, seq_len, hbm_bytes, headroom), 1)
    micro = train_batch_size // requested
    if micro > cap:
        return plan_batch_split(cfg, seq_len, train_batch_size, hbm_bytes, requested, headroom, merge=False), 1
    for passes in range(1, requested + 1):
        if requested % passes == 0 and (requested // passes) * micro <= cap:
            return requested, requested // passes
    return requested, 1


def device_hbm_bytes(device=None) -> Optional[int]:
    """Total HBM of the current (or given) GPU; None without one."""
    import torch
    if not torch.cuda.is_available():
        return None
    return torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device()).total_memory
