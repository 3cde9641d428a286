"""Rule-based English sentence splitter (stand-in for nltk's punkt model, which the reference loads
for ``--split_by_sentence``: ``split_dataset.py:230-244``; nltk is not installed here).

Splits after ``.``/``!``/``?`` (optionally followed by closing quotes/brackets) when the next token
starts like a sentence (upper-case letter, digit, opening quote/bracket or an HTML-ish tag as in the
NQ ``document_text``), except after common abbreviations and single-letter initials.
"""
from __future__ import annotations

import re
from typing import List

_ABBREV = {
    "mr", "mrs", "ms", "dr", "prof", "sr", "jr", "st", "vs", "etc", "inc", "ltd", "co", "corp", "jan", "feb",
    "mar", "apr", "jun", "jul", "aug", "sep", "sept", "oct", "nov", "dec", "no", "vol", "fig", "al", "e.g",
    "i.e", "u.s", "u.k", "gen", "gov", "lt", "col", "sgt", "capt", "rev", "mt", "ft", "approx", "dept", "est",
}
_END = re.compile(r"([.!?])([\"')\]]*)(\s+)(?=[A-Z0-9\"'(\[<])")


def split_sentences(text: str) -> List[str]:
    out = []
    start = 0
    for m in _END.finditer(text):
        end = m.end(2)
        prev = text[start:m.start(1)].split()
        last = prev[-1].lower().rstrip(".") if prev else ""
        if m.group(1) == "." and (last in _ABBREV or (len(last) == 1 and last.isalpha())):
            continue
        out.append(text[start:end])
        start = m.end(3)
    tail = text[start:]
    if tail.strip() or not out:
        out.append(tail)
    return out
