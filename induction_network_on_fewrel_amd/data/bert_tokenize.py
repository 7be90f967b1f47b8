"""BERT input features for FewRel instances (the north-star BERT encoder).

An instance ``{"tokens", "h": [name, qid, [[pos...], ...]], "t": ...}`` (reference data contract,
``util/data_loader.py:62-78``) becomes

    [CLS] w_0 ... [E1] head words [/E1] ... [E2] tail words [/E2] ... [SEP]

with entity-start markers (the standard FewRel BERT input: the sentence vector is the concatenation
of the hidden states at [E1] and [E2], or the [CLS] state).  Arrays per dataset (int32):
``ids [n, Lb]`` (0 = [PAD]), ``mask [n, Lb]`` (1 = real token), ``e1 / e2 [n]`` (marker positions,
clamped to Lb-1 after truncation), ``length [n]``.

Vocabulary: a BERT ``vocab.txt`` (WordPiece, greedy longest-match-first with ``##`` continuations;
markers use ``[unused0..3]`` when present) or, with no vocab file (no downloads are possible here),
a word-level vocabulary built from the data's own lower-cased tokens.
"""
from __future__ import annotations

import json
from collections import Counter, OrderedDict
from typing import Dict, Iterable, List, Optional

import numpy as np

SPECIALS = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
MARKERS = ["[E1]", "[/E1]", "[E2]", "[/E2]"]


class BertVocab:
    def __init__(self, tokens: List[str], wordpiece: bool, lower: bool = True):
        self.tokens = list(tokens)
        self.index: Dict[str, int] = {t: i for i, t in enumerate(self.tokens)}
        self.wordpiece = wordpiece
        self.lower = lower
        for t in SPECIALS:
            if t not in self.index:
                self._add(t)
        self.marker_ids = []
        for k, m in enumerate(MARKERS):
            unused = f"[unused{k}]"
            if m in self.index:
                self.marker_ids.append(self.index[m])
            elif unused in self.index:
                self.marker_ids.append(self.index[unused])
            else:
                self.marker_ids.append(self._add(m))
        self.pad, self.unk, self.cls, self.sep = (self.index[t] for t in ("[PAD]", "[UNK]", "[CLS]", "[SEP]"))

    def _add(self, t: str) -> int:
        self.index[t] = len(self.tokens)
        self.tokens.append(t)
        return self.index[t]

    def __len__(self) -> int:
        return len(self.tokens)

    # ------------------------------------------------------------------ builders
    @classmethod
    def from_vocab_file(cls, path: str, lower: bool = True) -> "BertVocab":
        with open(path, encoding="utf-8") as fh:
            toks = [line.rstrip("\n") for line in fh]
        return cls(toks, wordpiece=True, lower=lower)

    @classmethod
    def from_token_lists(cls, sents: Iterable[List[str]], max_size: int = 30522, min_count: int = 1,
                         lower: bool = True) -> "BertVocab":
        c = Counter()
        for toks in sents:
            c.update(t.lower() if lower else t for t in toks)
        base = SPECIALS + MARKERS
        words = [w for w, n in sorted(c.items(), key=lambda x: (-x[1], x[0])) if n >= min_count and w not in base]
        return cls(base + words[: max(0, max_size - len(base))], wordpiece=False, lower=lower)

    # ------------------------------------------------------------------ encoding
    def encode_word(self, w: str) -> List[int]:
        if self.lower:
            w = w.lower()
        if not self.wordpiece:
            return [self.index.get(w, self.unk)]
        if len(w) > 100:
            return [self.unk]
        out, start = [], 0
        while start < len(w):
            end, cur = len(w), None
            while start < end:
                piece = w[start:end] if start == 0 else "##" + w[start:end]
                if piece in self.index:
                    cur = self.index[piece]
                    break
                end -= 1
            if cur is None:
                return [self.unk]
            out.append(cur)
            start = end
        return out


def encode_instance(tokens: List[str], head: List[int], tail: List[int], vocab: BertVocab, max_length: int):
    """-> (ids list, e1, e2) for one instance (marker positions before truncation clamp)."""
    e1m, e1c, e2m, e2c = vocab.marker_ids
    seq = [vocab.cls]
    e1 = e2 = 0
    h0, h1, t0, t1 = head[0], head[-1], tail[0], tail[-1]
    for i, tok in enumerate(tokens):
        if i == h0:
            e1 = len(seq)
            seq.append(e1m)
        if i == t0:
            e2 = len(seq)
            seq.append(e2m)
        seq.extend(vocab.encode_word(tok))
        if i == h1:
            seq.append(e1c)
        if i == t1:
            seq.append(e2c)
    seq.append(vocab.sep)
    return seq, min(e1, max_length - 1), min(e2, max_length - 1)


def features_from_fewrel(ori_data: "OrderedDict[str, list]", vocab: BertVocab, max_length: int) -> Dict[str, np.ndarray]:
    """Instance order = relation order then instance order (the same order as FewRelDataset.tensorize)."""
    n = sum(len(v) for v in ori_data.values())
    ids = np.full((n, max_length), vocab.pad, dtype=np.int32)
    mask = np.zeros((n, max_length), dtype=np.int32)
    e1 = np.zeros((n,), dtype=np.int32)
    e2 = np.zeros((n,), dtype=np.int32)
    length = np.zeros((n,), dtype=np.int32)
    i = 0
    for _, items in ori_data.items():
        for ins in items:
            seq, a, b = encode_instance(ins["tokens"], ins["h"][2][0], ins["t"][2][0], vocab, max_length)
            if len(seq) > max_length:           # truncate, keep the closing [SEP]
                seq = seq[: max_length - 1] + [vocab.sep]
            ids[i, : len(seq)] = seq
            mask[i, : len(seq)] = 1
            e1[i], e2[i], length[i] = a, b, len(seq)
            i += 1
    return {"ids": ids, "mask": mask, "e1": e1, "e2": e2, "length": length}


def features_from_json(path: str, max_length: int, vocab: Optional[BertVocab] = None,
                       vocab_file: str = "") -> "tuple[Dict[str, np.ndarray], BertVocab]":
    with open(path, encoding="utf-8") as fh:
        ori = json.load(fh, object_pairs_hook=OrderedDict)
    if vocab is None:
        vocab = (BertVocab.from_vocab_file(vocab_file) if vocab_file else
                 BertVocab.from_token_lists(ins["tokens"] for items in ori.values() for ins in items))
    return features_from_fewrel(ori, vocab, max_length), vocab


def synthetic_features(data, vocab_size: int, max_length: int, seed: int = 0) -> Dict[str, np.ndarray]:
    """BERT features for a synthetic FewRelDataset: its word ids are folded into [9, vocab_size)
    and the entity markers are placed at the (first-token) entity positions the pos arrays encode."""
    n, L = data.data_word.shape
    base = len(SPECIALS) + len(MARKERS)
    ids = np.zeros((n, max_length), dtype=np.int32)
    mask = np.zeros((n, max_length), dtype=np.int32)
    e1 = np.zeros((n,), dtype=np.int32)
    e2 = np.zeros((n,), dtype=np.int32)
    length = np.zeros((n,), dtype=np.int32)
    ph = L - data.data_pos1[:, 0]          # pos1[i, j] = j - p_head + L
    pt = L - data.data_pos2[:, 0]
    words = base + (data.data_word.astype(np.int64) % max(1, vocab_size - base))
    for i in range(n):
        ln = int(data.data_length[i])
        seq = [2]
        for j in range(ln):
            if j == ph[i]:
                e1[i] = len(seq)
                seq.append(len(SPECIALS))          # [E1]
            if j == pt[i]:
                e2[i] = len(seq)
                seq.append(len(SPECIALS) + 2)      # [E2]
            seq.append(int(words[i, j]))
        seq.append(3)
        seq = seq[: max_length - 1] + [3] if len(seq) > max_length else seq
        ids[i, : len(seq)] = seq
        mask[i, : len(seq)] = 1
        length[i] = len(seq)
        e1[i] = min(e1[i], max_length - 1)
        e2[i] = min(e2[i], max_length - 1)
    return {"ids": ids, "mask": mask, "e1": e1, "e2": e2, "length": length}
