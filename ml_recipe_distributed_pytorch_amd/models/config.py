"""Architecture presets (the HF configs the reference pulls with ``from_pretrained``,
``modules/model/model/model.py:20-25``).  No network here, so the shapes are built in."""
from __future__ import annotations

from dataclasses import dataclass, replace


@dataclass
class EncoderConfig:
    family: str = "bert"            # bert | roberta
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    pad_token_id: int = 0
    unk_token_id: int = 100
    cls_token_id: int = 101
    sep_token_id: int = 102
    num_labels: int = 5

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def position_offset(self) -> int:
        """RoBERTa positions start at pad_token_id + 1 (HF create_position_ids_from_input_ids)."""
        return self.pad_token_id + 1 if self.family == "roberta" else 0


_BERT_BASE = EncoderConfig()
_BERT_LARGE = replace(_BERT_BASE, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                      intermediate_size=4096)
_ROBERTA_BASE = replace(_BERT_BASE, family="roberta", vocab_size=50265, max_position_embeddings=514,
                        type_vocab_size=1, pad_token_id=1, unk_token_id=3, cls_token_id=0, sep_token_id=2,
                        layer_norm_eps=1e-5)
_ROBERTA_LARGE = replace(_ROBERTA_BASE, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                         intermediate_size=4096)

PRESETS = {
    "bert-base-uncased": _BERT_BASE,
    "bert-base-cased": replace(_BERT_BASE, vocab_size=28996),
    "bert-large-uncased": _BERT_LARGE,
    "bert-large-cased": replace(_BERT_LARGE, vocab_size=28996),
    "roberta-base": _ROBERTA_BASE,
    "roberta-large": _ROBERTA_LARGE,
    # tiny shapes for fast tests; head_dim stays 64 so it runs the same HIP attention kernel
    "bert-tiny-test": replace(_BERT_BASE, vocab_size=1024, hidden_size=128, num_hidden_layers=2,
                              num_attention_heads=2, intermediate_size=256),
}


def get_config(name: str, **overrides) -> EncoderConfig:
    if name not in PRESETS:
        raise ValueError(f"Unknown model {name!r}; choices: {sorted(PRESETS)}")
    cfg = replace(PRESETS[name])
    for k, v in overrides.items():
        if v is not None:
            setattr(cfg, k, v)
    return cfg
