#!/usr/bin/env python3
"""No-training control through the SAME pipeline as the learned model (README "Accuracy", verdict r3 #7).

The learned encoders stay below a lexical TF-IDF baseline on relations unseen in training, and fold 2 is at
chance for every learned configuration.  This control separates "the encoder destroys the lexical signal"
from "the data is too small": it uses exactly what a training run sees --

* the tensorised val.json of ``train.py --split_val true --vocab_from_data true`` (same word table: random
  ``--dim``-d vectors per lower-cased token, seed = Config.seed, L2-normalised rows; UNK / BLANK zero);
* the held-out relations of ``train.py --fold k`` (relations 5k .. 5k+4, JSON order, wrapping);
* episodes from the reference-layout sampler (data/sampler.py::EpisodeSampler, support class-major, Q=5);

and replaces the trained encoder + induction + relation modules by: sentence vector = mean of its frozen word
vectors over the valid tokens (mask > 0), class prototype = mean of its K support vectors, prediction =
nearest prototype by cosine similarity.  Nothing is trained.

usage: python tools/control_baseline.py [--val gpudata/val.json] [--dims 50,300] [--folds 0,1,2] [--episodes 3000]
Prints one JSON line per (dim, fold, K) and a summary line per (dim, K).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _meanpool_accuracy(ds, W, K, episodes, seed, N=5, Q=5):
    """Mean of the frozen word vectors over the valid tokens -> nearest class prototype (cosine)."""
    from induction_network_on_fewrel_amd.data import EpisodeSampler
    valid = (ds.data_mask > 0).astype(np.float32)
    vec = (W[ds.data_word] * valid[..., None]).sum(1) / np.maximum(valid.sum(1, keepdims=True), 1.0)
    vec /= np.maximum(np.linalg.norm(vec, axis=1, keepdims=True), 1e-12)
    s = EpisodeSampler(ds, seed=seed)
    idx, labels = s.next_batch_indices(episodes, N, K, Q)
    sup = vec[idx[:, : N * K]].reshape(episodes, N, K, -1).mean(2)
    sup /= np.maximum(np.linalg.norm(sup, axis=-1, keepdims=True), 1e-12)
    pred = np.einsum("bqd,bnd->bqn", vec[idx[:, N * K:]], sup).argmax(-1)
    return float((pred == labels).mean())


def main():
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import EpisodeSampler, FewRelDataset, vocab_from_fewrel
    ap = argparse.ArgumentParser()
    ap.add_argument("--val", default=os.path.join(ROOT, "gpudata", "val.json"))
    ap.add_argument("--dims", default="50,300")
    ap.add_argument("--folds", default="0,1,2")
    ap.add_argument("--shots", default="1,5")
    ap.add_argument("--episodes", type=int, default=3000)
    ap.add_argument("--out", default="")
    ap.add_argument("--task", default="val", choices=["val", "transfer"],
                    help="transfer: the synthetic relation-transfer task's held-out test relations "
                         "(data/synthetic.py::make_transfer_splits with train.py's --synthetic_task transfer defaults)")
    ap.add_argument("--relations", type=int, default=48, help="transfer: training relations (--synthetic_relations)")
    ap.add_argument("--instances", type=int, default=300, help="transfer: instances per relation")
    ap.add_argument("--vocab", type=int, default=20000, help="transfer: --synthetic_vocab")
    ap.add_argument("--seed", type=int, default=None, help="transfer: --seed (default Config.seed)")
    args = ap.parse_args()
    cfg = Config()
    rows = []
    if args.task == "transfer":
        from induction_network_on_fewrel_amd.data.synthetic import make_transfer_splits
        seed = cfg.seed if args.seed is None else args.seed
        for dim in (int(x) for x in args.dims.split(",")):
            _, va, te = make_transfer_splits(args.relations, cfg.synthetic_val_relations, cfg.synthetic_test_relations,
                                             args.instances, cfg.max_length, args.vocab, dim, seed=seed)
            for split in (va, te):
                for K in (int(x) for x in args.shots.split(",")):
                    acc = _meanpool_accuracy(split, split.word_vec_mat, K, args.episodes, cfg.seed)
                    r = dict(control="meanpool-nearest-prototype", task="transfer", split=split.name, dim=dim, N=5,
                             K=K, episodes=args.episodes, relations=split.relations(), accuracy=round(acc, 4))
                    rows.append(r)
                    print(json.dumps(r), flush=True)
        if args.out:
            with open(args.out, "w") as fh:
                for r in rows:
                    fh.write(json.dumps(r) + "\n")
        return
    for dim in (int(x) for x in args.dims.split(",")):
        # the word table train.py --vocab_from_data builds (processed-data cache bypassed: written to /tmp)
        wv = f"/tmp/ina_control_vocab_{dim}.json"
        if not os.path.exists(wv):
            with open(wv, "w") as fh:
                json.dump(vocab_from_fewrel(args.val, dim=dim, seed=cfg.seed), fh)
        full = FewRelDataset.from_json(args.val, wv, cfg.max_length, cfg.case_sensitive,
                                       processed_dir=f"/tmp/ina_control_processed_{dim}")
        rels = full.relations()
        W = full.word_vec_mat
        for fold in (int(x) for x in args.folds.split(",")):
            test = [rels[(5 * fold + i) % len(rels)] for i in range(5)]
            te = full.subset_relations(test, "control")
            valid = (te.data_mask > 0).astype(np.float32)
            vec = (W[te.data_word] * valid[..., None]).sum(1) / np.maximum(valid.sum(1, keepdims=True), 1.0)
            vec /= np.maximum(np.linalg.norm(vec, axis=1, keepdims=True), 1e-12)
            for K in (int(x) for x in args.shots.split(",")):
                N, Q = 5, 5
                s = EpisodeSampler(te, seed=cfg.seed + fold)
                idx, labels = s.next_batch_indices(args.episodes, N, K, Q)   # [B, N K + N Q], [B, N Q]
                sup = vec[idx[:, : N * K]].reshape(args.episodes, N, K, -1).mean(2)
                sup /= np.maximum(np.linalg.norm(sup, axis=-1, keepdims=True), 1e-12)
                qry = vec[idx[:, N * K:]]
                pred = np.einsum("bqd,bnd->bqn", qry, sup).argmax(-1)
                acc = float((pred == labels).mean())
                r = dict(control="meanpool-nearest-prototype", dim=dim, fold=fold, N=N, K=K, episodes=args.episodes,
                         relations=test, accuracy=round(acc, 4))
                rows.append(r)
                print(json.dumps(r), flush=True)
    for dim in sorted({r["dim"] for r in rows}):
        for K in sorted({r["K"] for r in rows}):
            a = [r["accuracy"] for r in rows if r["dim"] == dim and r["K"] == K]
            print(json.dumps(dict(summary=f"{dim}-d 5-way {K}-shot", folds=[round(100 * x, 1) for x in a],
                                  mean=round(100 * float(np.mean(a)), 1), std=round(100 * float(np.std(a)), 1))))
    if args.out:
        with open(args.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
