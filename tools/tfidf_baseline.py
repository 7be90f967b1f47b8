#!/usr/bin/env python3
"""No-training lexical baseline for the val.json splits: TF-IDF bag-of-words nearest prototype.

Puts the learned models' accuracy in context (README "Accuracy"): on the relation-disjoint split it
uses the same held-out relations as ``train.py --split_val true --train_relations 11`` (JSON order);
``--instance`` mirrors ``--split_mode instance`` (prototypes and queries from the last 30% of each
relation).  Episodes: N-way K-shot, 5 queries per class, 2000 episodes.

usage: python tools/tfidf_baseline.py [--val gpudata/val.json] [--train_relations 11] [--instance] [--fold k]
(--fold k: the held-out relations of ``train.py --fold k``, relations 5k .. 5k+4 in JSON order, wrapping)
"""
import argparse
import collections
import json
import random

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--val", default="gpudata/val.json")
    ap.add_argument("--train_relations", type=int, default=11)
    ap.add_argument("--instance", action="store_true")
    ap.add_argument("--episodes", type=int, default=2000)
    ap.add_argument("--fold", type=int, default=-1)
    args = ap.parse_args()
    d = json.load(open(args.val))
    rels = list(d.keys())
    if args.instance:
        test = rels
        pools = {r: d[r][int(round(0.7 * len(d[r]))):] for r in rels}
    else:
        test = ([rels[(5 * args.fold + i) % len(rels)] for i in range(5)] if args.fold >= 0
                else rels[args.train_relations:])
        pools = {r: d[r] for r in test}
    docs = {r: [[t.lower() for t in x["tokens"]] for x in d[r]] for r in rels}
    df = collections.Counter()
    for r in rels:
        for toks in docs[r]:
            df.update(set(toks))
    n_docs = sum(len(v) for v in docs.values())
    vocab = {w: i for i, w in enumerate(df)}
    idf = np.array([np.log(n_docs / (1 + df[w])) for w in vocab])

    def vec(toks):
        v = np.zeros(len(vocab))
        for t in toks:
            v[vocab[t.lower()]] += 1
        v *= idf
        return v / (np.linalg.norm(v) + 1e-9)

    V = {r: np.stack([vec(x["tokens"]) for x in pools[r]]) for r in test}
    random.seed(0)
    np.random.seed(0)
    for K in (1, 5):
        acc = []
        for _ in range(args.episodes):
            cl = random.sample(test, 5)
            protos, qs, ql = [], [], []
            for i, r in enumerate(cl):
                idx = np.random.choice(len(V[r]), K + 5, replace=False)
                protos.append(V[r][idx[:K]].mean(0))
                qs.append(V[r][idx[K:]])
                ql += [i] * 5
            P, Qm = np.stack(protos), np.concatenate(qs)
            acc.append(((Qm @ P.T).argmax(1) == np.array(ql)).mean())
        print(json.dumps({"split": "instance" if args.instance else "relation", "fold": args.fold, "way": 5, "shot": K,
                          "accuracy": round(float(np.mean(acc)), 4)}))


if __name__ == "__main__":
    main()
