"""Synthetic FewRel-shaped data (benchmarks and tests run on synthetic tokens).

Shapes follow the measured val.json statistics (L=37, ~33% padding): sentence lengths are
drawn from val.json's length histogram (6..36 tokens, mean 24.8; ``length_dist="uniform"`` gives the
round-1/2 uniform 6..36 draw, mean 21). Each relation owns a few "trigger" tokens placed between the
two entities so that the task is learnable (integration tests check that accuracy rises above chance).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .fewrel import FewRelDataset


# instances per token length in the reference's data/val.json (lengths 6..36; 11,200 instances)
FEWREL_VAL_LENGTH_HIST = {6: 2, 7: 7, 8: 18, 9: 22, 10: 52, 11: 156, 12: 216, 13: 158, 14: 226, 15: 260, 16: 275,
                          17: 343, 18: 355, 19: 424, 20: 429, 21: 485, 22: 567, 23: 566, 24: 574, 25: 578, 26: 596,
                          27: 602, 28: 618, 29: 586, 30: 550, 31: 537, 32: 507, 33: 447, 34: 360, 35: 343, 36: 341}


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
                   with_word_vectors: bool = True, length_dist: str = "fewrel") -> FewRelDataset:
    rng = np.random.default_rng(seed)
    L = max_length
    R, I = num_relations, instances_per_relation
    tot = R * I
    unk, blank = vocab, vocab + 1
    max_len = min(max_len, L)
    min_len = max(1, min(min_len, max_len))
    if length_dist == "fewrel":
        ls = np.array([k for k in FEWREL_VAL_LENGTH_HIST if min_len <= k <= max_len], dtype=np.int32)
        if len(ls) == 0:   # a max_length below FewRel's shortest sentence: every row full length
            lengths = np.full(tot, max_len, dtype=np.int32)
        else:
            w = np.array([FEWREL_VAL_LENGTH_HIST[k] for k in ls], dtype=np.float64)
            lengths = rng.choice(ls, size=tot, p=w / w.sum()).astype(np.int32)
    elif length_dist == "uniform":
        lengths = rng.integers(min_len, max_len + 1, size=tot).astype(np.int32)
    else:
        raise ValueError(f"unknown length_dist {length_dist}")
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


def make_transfer_splits(train_relations: int = 48, val_relations: int = 8, test_relations: int = 8,
                         instances_per_relation: int = 300, max_length: int = 37, vocab: int = 20000,
                         word_dim: int = 50, triggers_per_relation: int = 4, triggers_in_span: int = 2,
                         distractors: int = 4, min_gap: int = 3, max_gap: int = 7, seed: int = 0):
    """Few-shot RELATION-TRANSFER task (verdict r4 #5): three relation-disjoint splits (train / val / test)
    whose relations the encoder can only tell apart by what lies BETWEEN the two entities.

    * Relation r owns ``triggers_per_relation`` trigger tokens (disjoint across ALL relations of all splits,
      so val / test relations bring trigger tokens never seen in training).
    * A sentence (length from val.json's histogram) has head / tail entities ``min_gap .. max_gap`` tokens
      apart (random order); ``triggers_in_span`` of r's triggers sit between them, the rest of the span is
      filler.
    * Outside the span sit ``distractors`` triggers of OTHER relations of the same split -- in a test episode
      often of the episode's other classes -- plus filler.  A bag of words (mean-pooled word vectors:
      tools/control_baseline.py --task transfer) therefore sees more wrong-class than right-class triggers;
      a model that learned (on the training relations) to read the span between the entities through the
      position features transfers to the unseen relations.
    -> (train, val, test) FewRelDatasets sharing one frozen random word table (``word_dim``-d)."""
    rng = np.random.default_rng(seed)
    L = max_length
    R = train_relations + val_relations + test_relations
    T = triggers_per_relation
    if R * T >= vocab // 2:
        raise ValueError("vocab too small for the trigger tokens")
    mat = random_word_vectors(vocab, word_dim, seed + 1)
    w2i = transfer_vocab(vocab)
    bounds = np.cumsum([0, train_relations, val_relations, test_relations])
    out = []
    for part, name in enumerate(("train", "val", "test")):
        rels = np.arange(bounds[part], bounds[part + 1])
        word, pos1, pos2, mask, lengths, _, _ = _transfer_part(
            rng, rels, instances_per_relation, L, vocab, T, triggers_in_span, distractors, min_gap, max_gap,
            (R * T, vocab))
        rel2scope = OrderedDict((f"T{r}", [k * instances_per_relation, (k + 1) * instances_per_relation])
                                for k, r in enumerate(rels))
        out.append(FewRelDataset(word, pos1, pos2, mask, lengths, rel2scope, mat, w2i, f"transfer_{name}"))
    return tuple(out)


def transfer_vocab(vocab: int) -> dict:
    """The synthetic tasks' token strings: id i <-> "w<i>" (so a generated split can be written as FewRel JSON and
    read back through --test_file with the training vocabulary)."""
    w2i = {f"w{i}": i for i in range(vocab)}
    w2i["UNK"], w2i["BLANK"] = vocab, vocab + 1
    return w2i


def _transfer_part(rng, rels, I, L, vocab, T, triggers_in_span, distractors, min_gap, max_gap, filler):
    """One relation split of the transfer task: sentences of relation r carry ``triggers_in_span`` of r's trigger
    tokens (ids r T .. r T + T - 1) between the entities and ``distractors`` triggers of the split's other relations
    outside them; filler tokens are uniform over ``filler`` = [lo, hi).  -> (word, pos1, pos2, mask, lengths, p1, p2)."""
    blank = vocab + 1
    ls_all = np.array([k for k in FEWREL_VAL_LENGTH_HIST if max_gap + 4 <= k <= min(36, L)], dtype=np.int32)
    w_all = np.array([FEWREL_VAL_LENGTH_HIST[k] for k in ls_all], dtype=np.float64)
    nr = len(rels)
    tot = nr * I
    lengths = rng.choice(ls_all, size=tot, p=w_all / w_all.sum()).astype(np.int32)
    word = rng.integers(filler[0], filler[1], size=(tot, L)).astype(np.int32)   # filler (never a trigger)
    p1 = np.zeros(tot, dtype=np.int32)
    p2 = np.zeros(tot, dtype=np.int32)
    for i in range(tot):
        r = rels[i // I]
        n = lengths[i]
        gap = int(rng.integers(min_gap, max_gap + 1))
        a = int(rng.integers(0, n - gap - 1))
        b = a + gap + 1
        if rng.random() < 0.5:
            p1[i], p2[i] = a, b
        else:
            p1[i], p2[i] = b, a
        span = np.arange(a + 1, b)
        for pos in rng.choice(span, size=min(triggers_in_span, len(span)), replace=False):
            word[i, pos] = r * T + int(rng.integers(0, T))
        outside = np.concatenate([np.arange(0, a), np.arange(b + 1, n)])
        others = rels[rels != r]
        if len(others) and len(outside):
            for pos in rng.choice(outside, size=min(distractors, len(outside)), replace=False):
                word[i, pos] = int(rng.choice(others)) * T + int(rng.integers(0, T))
    j = np.arange(L, dtype=np.int32)[None, :]
    word[j >= lengths[:, None]] = blank
    pos1 = (j - p1[:, None] + L).astype(np.int32)
    pos2 = (j - p2[:, None] + L).astype(np.int32)
    lo = np.minimum(p1, p2)[:, None]
    hi = np.maximum(p1, p2)[:, None]
    mask = np.where(j <= lo, 1, np.where(j <= hi, 2, 3)).astype(np.int32)
    mask[j >= lengths[:, None]] = 0
    return word, pos1, pos2, mask, lengths, p1, p2


def write_shifted_transfer_json(path: str, relations: int = 8, instances_per_relation: int = 300,
                                max_length: int = 37, vocab: int = 20000, triggers_per_relation: int = 4,
                                first_relation: int = 64, triggers_in_span: int = 2, distractors: int = 6,
                                min_gap: int = 5, max_gap: int = 11, seed: int = 7) -> str:
    """A DOMAIN-SHIFTED test set for the transfer task, written as FewRel JSON (tokens "w<id>", entities by first
    token position) for ``fewrel_eval.py --test_file`` / ``train.py --test_file`` (FewRel 2.0 domain adaptation:
    BASELINE.json config 5).  Against make_transfer_splits' test split it changes the generator:
      * new relations (``first_relation`` ..: trigger tokens never seen in training, validation or testing),
      * entity gaps of ``min_gap`` .. ``max_gap`` tokens (training: 3 .. 7) -> longer spans, more filler inside,
      * ``distractors`` other-class triggers outside the span (training: 4),
      * filler words from the upper half of the filler vocabulary only (a shifted word distribution);
    the word table (and so the vocabulary) is the training one."""
    import json
    rng = np.random.default_rng(seed)
    T = triggers_per_relation
    rels = np.arange(first_relation, first_relation + relations)
    if (first_relation + relations) * T >= vocab // 2:
        raise ValueError("vocab too small for the trigger tokens")
    word, _, _, _, lengths, p1, p2 = _transfer_part(rng, rels, instances_per_relation, max_length, vocab, T,
                                                    triggers_in_span, distractors, min_gap, max_gap,
                                                    ((vocab // 2 + vocab) // 2, vocab))
    out = OrderedDict()
    for k, r in enumerate(rels):
        items = []
        for i in range(k * instances_per_relation, (k + 1) * instances_per_relation):
            n = int(lengths[i])
            toks = [f"w{int(t)}" for t in word[i, :n]]
            items.append({"tokens": toks, "h": [toks[p1[i]], "Qh", [[int(p1[i])]]],
                          "t": [toks[p2[i]], "Qt", [[int(p2[i])]]]})
        out[f"S{int(r)}"] = items
    with open(path, "w") as fh:
        json.dump(out, fh)
    return path



if __name__ == "__main__":   # python -m induction_network_on_fewrel_amd.data.synthetic --shifted_test out.json
    import argparse
    ap = argparse.ArgumentParser(description="write the transfer task's domain-shifted test set (FewRel JSON)")
    ap.add_argument("--shifted_test", required=True)
    ap.add_argument("--relations", type=int, default=8)
    ap.add_argument("--instances", type=int, default=300)
    ap.add_argument("--vocab", type=int, default=20000)
    ap.add_argument("--first_relation", type=int, default=64, help=">= train + val + test relations of the task")
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    print(write_shifted_transfer_json(a.shifted_test, a.relations, a.instances, vocab=a.vocab,
                                      first_relation=a.first_relation, seed=a.seed))
