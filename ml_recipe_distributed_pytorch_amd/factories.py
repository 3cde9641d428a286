"""Component factories (reference ``modules/init.py:18-205``): loss, model+tokenizer, optimizer,
datasets, collate function.

Environment gaps handled here: no network, so pretrained weights come from ``--pretrained_path``
(random init otherwise) and the tokenizer from ``--vocab_file``/``--merges_file`` (the dummy path
needs neither: special ids come from the model preset).  ``transformers.AdamW`` no longer exists, so
the optimizer is our fused HF-semantics AdamW (D18); the ``'robrta'`` typo fallback is fixed (D10).
"""
from __future__ import annotations

import functools
import logging
import os
from collections import defaultdict
from typing import Optional

import numpy as np
import torch

from .data.collate import collate_fun
from .data.dummy import DummyDataset, SpecialIds
from .data.items import LABELS, LABELS2ID
from .models.bert import BertForQuestionAnswering, load_pretrained
from .models.config import get_config
from .models.losses import build_loss
from .train.optim import FusedAdaMod, FusedAdamW
from .train.trainer import optimizer_groups

logger = logging.getLogger(__name__)


def init_loss(params, train_weights=None):
    loss = build_loss(params, train_weights, n_classes=len(LABELS))
    logger.info(f"Used loss function for classification: {type(loss._losses['cls'][0]).__name__}.")
    return loss


def init_tokenizer(model_params, *, bpe_dropout=None):
    from .data.tokenizer import Tokenizer
    family = "roberta" if model_params.model.startswith("roberta") else "bert"
    vocab = getattr(model_params, "vocab_file", None)
    if vocab is not None and os.path.exists(vocab):
        return Tokenizer(model_name=family, vocab_file=vocab, merges_file=getattr(model_params, "merges_file", None),
                         lowercase=getattr(model_params, "lowercase", True),
                         handle_chinese_chars=getattr(model_params, "handle_chinese_chars", False),
                         dropout=bpe_dropout, legacy=getattr(model_params, "legacy_tokenization", False))
    cfg = get_config(model_params.model)
    logger.warning("No vocab file: using the preset special ids only (sufficient for --dummy_dataset; "
                   "real NQ preprocessing needs --vocab_file).")
    return SpecialIds(cfg.vocab_size, cfg.pad_token_id, cfg.unk_token_id, cfg.cls_token_id, cfg.sep_token_id, family)


def init_model(model_params, *, checkpoint=None, device=torch.device("cpu"), bpe_dropout=None, seed=None,
               precision: Optional[str] = None):
    model_params.model_name = "roberta" if model_params.model.startswith("roberta") else "bert"
    tokenizer = init_tokenizer(model_params, bpe_dropout=bpe_dropout)
    cfg = get_config(model_params.model, hidden_dropout_prob=model_params.hidden_dropout_prob,
                     attention_probs_dropout_prob=model_params.attention_probs_dropout_prob,
                     layer_norm_eps=model_params.layer_norm_eps)
    if hasattr(tokenizer, "__len__") and len(tokenizer) > cfg.vocab_size:
        cfg.vocab_size = len(tokenizer)
    prec = precision or ("bf16" if torch.device(device).type == "cuda" else "fp32")
    model = BertForQuestionAnswering(cfg, precision=prec, seed=seed)
    pre = getattr(model_params, "pretrained_path", None)
    if pre and getattr(model_params, "random_init", False):
        logger.warning(f"--random_init: ignoring --pretrained_path {pre}.")
        pre = None
    if pre:
        missing = load_pretrained(model, pre)
        logger.info(f"Pretrained encoder weights loaded from {pre} ({len(missing)} tensors left at init).")
    else:
        logger.warning("No --pretrained_path: encoder is randomly initialised (no network in this environment).")
    model.to(device)
    if checkpoint is not None:
        state = torch.load(checkpoint, map_location="cpu", weights_only=True)
        model.load_state_dict(state["model"], strict=False)
        logger.info(f"Model checkpoint was restored from {checkpoint}.")
    return model, tokenizer


def _optimized_parameters(params, model):
    if getattr(params, "finetune", False):
        if params.apex_level is not None:
            params.apex_level = None
            logger.warning("Finetune mode is not supported with Apex.")
        model.eval()
        modules, named = [], []
        sel = [("finetune_transformer", ["transformer"]), ("finetune_position", ["position_outputs"]),
               ("finetune_position_reg", ["reg_start", "reg_end"]), ("finetune_class", ["classifier"])]
        for flag, names in sel:
            if getattr(params, flag, False):
                for n in names:
                    modules.append(getattr(model, n))
                    named.extend((f"{n}.{k}", p) for k, p in modules[-1].named_parameters())
        if not modules:
            raise AttributeError("Specify at least one module for fine-tuning.")
        trainable = {id(p) for _, p in named}
        for p in model.parameters():
            p.requires_grad_(id(p) in trainable)
        logger.info(f"Fine-tuned modules: transformer({params.finetune_transformer}), "
                    f"position({params.finetune_position}), classifier({params.finetune_class}).")
        return modules, named
    return None, list(model.named_parameters())


def init_optimizer(params, model):
    modules, named = _optimized_parameters(params, model)
    groups = optimizer_groups(named, params.weight_decay)
    groups = [g for g in groups if g["params"]]
    if params.optimizer == "adam":
        opt = FusedAdamW(groups, model.store, lr=params.lr, eps=1e-6, correct_bias=False, zero_grad_fn=model.zero_grad)
    else:
        opt = FusedAdaMod(groups, model.store, lr=params.lr, zero_grad_fn=model.zero_grad)
    logger.info(f"Used optimizer: {type(opt).__name__}.")
    if modules is not None:
        model.list_of_trainable_modules = modules
    return opt


def init_datasets(params, *, tokenizer=None, clear=False, rank: int = -1):
    weights = defaultdict(lambda: None)
    common = dict(max_seq_len=params.max_seq_len, max_question_len=params.max_question_len,
                  doc_stride=params.doc_stride, split_by_sentence=params.split_by_sentence, truncate=params.truncate)
    if params.dummy_dataset:
        logger.warning("Dummy dataset is used to train model.")
        n = getattr(params, "dummy_dataset_len", 10000)
        train = DummyDataset(tokenizer, dataset_len=n, **common)
        test = DummyDataset(tokenizer, dataset_len=n, **common) if rank in (-1, 0) or getattr(params, "eval_shard", False) else None
        return train, test, weights
    from .data.nq import RawPreprocessor, SplitDataset
    pre = RawPreprocessor(raw_json=params.data_path, out_dir=params.processed_data_path, clear=clear)
    labels_counter, labels, (train_idx, train_labels, test_idx, test_labels) = pre()
    if getattr(params, "train_label_weights", False):
        lw = np.asarray([1.0 / labels_counter[k] for k in sorted(labels_counter.keys())])
        lw = lw / lw.sum()
        logger.info("Label weights: " + ", ".join(f"{LABELS[k]} ({k}) - {v:.4f}" for k, v in enumerate(lw)))
        weights["label_weights"] = torch.from_numpy(lw)
    if getattr(params, "train_sampler_weights", False):
        sw = np.asarray([1.0 / labels_counter[int(l)] for l in train_labels])
        weights["sampler_weights"] = sw / sw.sum()
    train = SplitDataset(params.processed_data_path, tokenizer, train_idx, **common)
    test = SplitDataset(params.processed_data_path, tokenizer, test_idx, test=True, **common) \
        if rank in (-1, 0) or getattr(params, "eval_shard", False) else None
    return train, test, weights


def init_collate_fun(tokenizer, return_items=False):
    return functools.partial(collate_fun, tokenizer=tokenizer, return_items=return_items)
