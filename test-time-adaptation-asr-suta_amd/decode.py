"""Greedy CTC decode and corpus WER (host side, reference row f1).

decode: Wav2Vec2CTCTokenizer.batch_decode of argmax ids as main.py:333-334 uses it
        (HF tokenization_wav2vec2.py:297-340, 411-450): group repeated ids, drop the pad/blank
        id 0, map the word delimiter '|' to a space, strip.
wer:    jiwer.wer(truth, hypothesis) (main.py:336, 408-434) restated: word-level Levenshtein
        after jiwer's default transform (collapse whitespace, strip, split on spaces), corpus
        WER = sum of (S + D + I) over pairs / sum of reference words.
"""
from __future__ import annotations

import re
from typing import List, Sequence, Tuple

import numpy as np

# facebook/wav2vec2-base-960h vocabulary (the reference ships the same table as vocab.json)
VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "E", "T", "A", "O", "N", "I", "H", "S", "R", "D", "L", "U", "M",
         "W", "C", "F", "G", "Y", "P", "B", "V", "K", "'", "X", "J", "Q", "Z"]
PAD_ID = 0
WORD_DELIM = "|"


def ctc_decode(ids: Sequence[int], vocab: Sequence[str] = VOCAB) -> str:
    """group repeats -> drop pad -> '|' to ' ' -> join -> strip (special tokens kept verbatim)."""
    out: List[str] = []
    prev = None
    for i in ids:
        i = int(i)
        if i == prev:
            continue
        prev = i
        if i == PAD_ID:
            continue
        tok = vocab[i] if 0 <= i < len(vocab) else "<unk>"
        out.append(" " if tok == WORD_DELIM else tok)
    return "".join(out).strip()


def batch_decode(ids: np.ndarray) -> List[str]:
    ids = np.asarray(ids)
    if ids.ndim == 1:
        ids = ids[None]
    return [ctc_decode(r) for r in ids]


def _words(s: str) -> List[str]:
    """jiwer wer_default: RemoveMultipleSpaces, Strip, ReduceToListOfListOfWords."""
    s = re.sub(r"\s\s+", " ", s).strip()
    return [w for w in s.split(" ") if len(w) >= 1]


def edit_distance(ref: Sequence[str], hyp: Sequence[str]) -> int:
    """Levenshtein distance over word lists (S, D, I unit costs)."""
    n, m = len(ref), len(hyp)
    if n == 0:
        return m
    if m == 0:
        return n
    prev = list(range(m + 1))
    for i in range(1, n + 1):
        cur = [i] + [0] * m
        ri = ref[i - 1]
        for j in range(1, m + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ri != hyp[j - 1]))
        prev = cur
    return prev[m]


def wer_counts(truth: Sequence[str], hyp: Sequence[str]) -> Tuple[int, int]:
    """(total edits, total reference words) over sentence pairs."""
    if len(truth) != len(hyp):
        raise ValueError("truth and hypothesis lists differ in length")
    e = w = 0
    for t, h in zip(truth, hyp):
        tw = _words(t)
        if not tw:
            raise ValueError("one or more references are empty strings")  # jiwer raises too
        e += edit_distance(tw, _words(h))
        w += len(tw)
    return e, w


def wer(truth, hyp) -> float:
    if isinstance(truth, str):
        truth = [truth]
    if isinstance(hyp, str):
        hyp = [hyp]
    e, w = wer_counts(list(truth), list(hyp))
    return e / w
