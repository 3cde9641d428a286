"""Tokenizer wrapper (reference ``modules/model/model/tokenizer.py:8-93``) over the native C++ WordPiece
(BERT) and byte-level BPE (RoBERTa) in ``_hq_host`` — replaces the Rust HF ``tokenizers`` dependency.

Deliberate fix of reference quirk D11: ``encode(text)`` returns ids WITHOUT special tokens (the
reference's ``BertWordPieceTokenizer.encode`` wrapped every word in [CLS] … [SEP] because its
post-processor was active).  ``legacy=True`` (``--legacy_tokenization``) restores that behaviour.
"""
from __future__ import annotations

import logging
import os
from typing import List, Optional

from .._native import host

logger = logging.getLogger(__name__)


class Tokenizer:
    def __init__(self, model_name: str, vocab_file: str, *, merges_file: Optional[str] = None, lowercase: bool = True,
                 handle_chinese_chars: bool = False, dropout: Optional[float] = None, legacy: bool = False,
                 seed: int = 0):
        self._args = dict(model_name=model_name, vocab_file=vocab_file, merges_file=merges_file, lowercase=lowercase,
                          handle_chinese_chars=handle_chinese_chars, dropout=dropout, legacy=legacy, seed=seed)
        self.model_name = model_name
        self.legacy = legacy
        if model_name == "bert":
            self._pad_token, self._sep_token, self._cls_token, self._unk_token = "[PAD]", "[SEP]", "[CLS]", "[UNK]"
            if dropout is not None:
                logger.warning("BPE dropout is not supported by the WordPiece tokenizer.")
            self._tok = host().WordPiece(vocab_file, lowercase, -1, handle_chinese_chars, self._unk_token, 100)
        elif model_name == "roberta":
            if merges_file is None:
                raise AttributeError("To use ByteLevelTokenizer, specify path to merges file.")
            self._pad_token, self._sep_token, self._cls_token, self._unk_token = "<pad>", "</s>", "<s>", "<unk>"
            self._tok = host().ByteLevelBPE(vocab_file, merges_file, float(dropout or 0.0), seed)
        else:
            raise NotImplementedError(f"Tokenizer initialization for model {model_name} is not implemented.")

    def __getstate__(self):
        # the native tokenizer is rebuilt from its files: picklable for spawn/Pool workers (the
        # reference's validate swapped in the slow HF tokenizer for that reason, validate.py:38-40)
        return self._args

    def __setstate__(self, args):
        self.__init__(**args)

    def __len__(self):
        return len(self._tok)

    def encode(self, string: str) -> List[int]:
        ids = list(self._tok.encode(string))
        if self.legacy and self.model_name == "bert":
            ids = [self.cls_token_id] + ids + [self.sep_token_id]
        return ids

    def encode_batch(self, strings: List[str]) -> List[List[int]]:
        if self.model_name == "bert" and not self.legacy:
            return [list(x) for x in self._tok.encode_batch(list(strings))]
        return [self.encode(s) for s in strings]

    def decode(self, ids, *, skip_special_tokens: bool = True) -> str:
        specials = {self.pad_token_id, self.sep_token_id, self.cls_token_id} if skip_special_tokens else set()
        ids = [int(i) for i in ids if int(i) not in specials]
        if self.model_name == "bert":
            return " ".join(self._tok.id_to_token(i) for i in ids).replace(" ##", "")
        return self._tok.decode(ids)

    def token_to_id(self, token: str) -> Optional[int]:
        i = self._tok.token_to_id(token)
        return None if i < 0 else i

    @property
    def pad_token_id(self):
        return self.token_to_id(self._pad_token)

    @property
    def sep_token_id(self):
        return self.token_to_id(self._sep_token)

    @property
    def cls_token_id(self):
        return self.token_to_id(self._cls_token)

    @property
    def unk_token_id(self):
        return self.token_to_id(self._unk_token)

    @property
    def pad_token(self):
        return self._pad_token

    @property
    def sep_token(self):
        return self._sep_token

    @property
    def cls_token(self):
        return self._cls_token

    @property
    def unk_token(self):
        return self._unk_token
