"""Synthetic FewRel-shaped data (benchmarks and tests run on synthetic tokens).

Shapes follow the measured val.json statistics (length 6..36, L=37, ~33%
padding). Each relation owns a few "trigger" tokens placed between the two entities so
that the task is learnable (integration tests check that accuracy rises above chance).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .fewrel import FewRelDataset


def random_word_vectors(vocab: int, dim: int, seed: int = 0) -> np.ndarray:
    """[vocab + 2, dim] L2-normalised table with zero UNK/BLANK rows (data_loader.py:130-140)."""
    rng = np.random.default_rng(seed)
    mat = np.zeros((vocab + 2, dim), dtype=np.float32)
    v = rng.standard_normal((vocab, dim)).astype(np.float32)
    v /= np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-12)
    mat[:vocab] = v
    return mat


def make_synthetic(num_relations: int = 64, instances_per_relation: int = 700, max_length: int = 37,
                   vocab: int = 400000, word_dim: int = 5, min_len: int = 6, max_len: int = 36,
                   triggers_per_relation: int = 8, triggers_per_sentence: int = 3, seed: int = 0,
                   with_word_vectors: bool = True) -> FewRelDataset:
    rng = np.random.default_rng(seed)
    L = max_length
    R, I = num_relations, instances_per_relation
    tot = R * I
    unk, blank = vocab, vocab + 1
    max_len = min(max_len, L)
    min_len = max(1, min(min_len, max_len))
    lengths = rng.integers(min_len, max_len + 1, size=tot).astype(np.int32)
    word = rng.integers(0, vocab, size=(tot, L)).astype(np.int32)
    # a sprinkle of OOV tokens, like real text
    oov = rng.random((tot, L)) < 0.02
    word[oov] = unk
    triggers = rng.integers(0, vocab, size=(R, triggers_per_relation)).astype(np.int32)
    j = np.arange(L, dtype=np.int32)[None, :]
    p1 = (rng.random(tot) * lengths).astype(np.int32)
    p2 = (rng.random(tot) * lengths).astype(np.int32)
    p1 = np.minimum(p1, L - 1)
    p2 = np.minimum(p2, L - 1)
    rel_of = np.repeat(np.arange(R), I)
    for i in range(tot):
        n = lengths[i]
        tpos = rng.integers(0, n, size=triggers_per_sentence)
        word[i, tpos] = triggers[rel_of[i], rng.integers(0, triggers_per_relation, size=triggers_per_sentence)]
    word[j >= lengths[:, None]] = blank
    pos1 = (j - p1[:, None] + L).astype(np.int32)
    pos2 = (j - p2[:, None] + L).astype(np.int32)
    lo = np.minimum(p1, p2)[:, None]
    hi = np.maximum(p1, p2)[:, None]
    mask = np.where(j <= lo, 1, np.where(j <= hi, 2, 3)).astype(np.int32)
    mask[j >= lengths[:, None]] = 0
    rel2scope = OrderedDict((f"S{r}", [r * I, (r + 1) * I]) for r in range(R))
    mat = random_word_vectors(vocab, word_dim, seed + 1) if with_word_vectors else None
    return FewRelDataset(word, pos1, pos2, mask, lengths, rel2scope, mat, None, "synthetic")
