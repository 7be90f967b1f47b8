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


def _meanpool_scores(ds, W, K, episodes, seed, N=5, Q=5, nota_rate=0.0):
    """Mean of the frozen word vectors over the valid tokens -> cosine similarity of each query to each class
    prototype (mean of its K support vectors).  -> (scores [B, N Q, N], labels [B, N Q]; label N = NOTA)."""
    from induction_network_on_fewrel_amd.data import EpisodeSampler
    valid = (ds.data_mask > 0).astype(np.float32)
    vec = (W[ds.data_word] * valid[..., None]).sum(1) / np.maximum(valid.sum(1, keepdims=True), 1.0)
    vec /= np.maximum(np.linalg.norm(vec, axis=1, keepdims=True), 1e-12)
    s = EpisodeSampler(ds, seed=seed, nota_rate=nota_rate)
    idx, labels = s.next_batch_indices(episodes, N, K, Q)
    sup = vec[idx[:, : N * K]].reshape(episodes, N, K, -1).mean(2)
    sup /= np.maximum(np.linalg.norm(sup, axis=-1, keepdims=True), 1e-12)
    return np.einsum("bqd,bnd->bqn", vec[idx[:, N * K:]], sup), labels


def _predict(scores, thr, N):
    pred = scores.argmax(-1)
    return pred if thr is None else np.where(scores.max(-1) < thr, N, pred)


def _meanpool_accuracy(ds, W, K, episodes, seed, N=5, Q=5):
    """Nearest class prototype (cosine) accuracy."""
    scores, labels = _meanpool_scores(ds, W, K, episodes, seed, N, Q)
    return float((scores.argmax(-1) == labels).mean())


def _meanpool_nota(tune, test, W, K, episodes, seed, rate, N=5, Q=5):
    """FewRel 2.0 NOTA rule for the control, as runtime/evaluate.py does for the model: a query whose best score is
    below a threshold is NOTA; the threshold maximises accuracy on ``tune`` episodes (the validation relations)."""
    ts, tl = _meanpool_scores(tune, W, K, 500, seed + 1, N, Q, rate)
    grid = np.linspace(-1.0, 1.0, 201)
    accs = [float((_predict(ts, t, N) == tl).mean()) for t in grid]
    thr = float(grid[int(np.argmax(accs))])
    sc, lab = _meanpool_scores(test, W, K, episodes, seed, N, Q, rate)
    pred = _predict(sc, thr, N)
    nota, pn = lab == N, pred == N
    return dict(threshold=round(thr, 3), accuracy=round(float((pred == lab).mean()), 4),
                in_class_accuracy=round(float((pred == lab)[~nota].mean()), 4),
                nota_precision=round(float((pn & nota).sum()) / max(1, int(pn.sum())), 4),
                nota_recall=round(float((pn & nota).sum()) / max(1, int(nota.sum())), 4),
                nota_fraction=round(float(nota.mean()), 4))


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
    ap.add_argument("--nota_rates", default="", help="transfer: also the FewRel 2.0 NOTA rule at these rates "
                    "(threshold tuned on the validation relations), e.g. 0,0.15,0.5")
    ap.add_argument("--test_file", default="", help="transfer: also a domain-shifted FewRel JSON (e.g. "
                    "data/synthetic.py --shifted_test) tensorised with the task's vocabulary")
    args = ap.parse_args()
    cfg = Config()
    rows = []
    if args.task == "transfer":
        from induction_network_on_fewrel_amd.data.synthetic import make_transfer_splits
        seed = cfg.seed if args.seed is None else args.seed
        for dim in (int(x) for x in args.dims.split(",")):
            _, va, te = make_transfer_splits(args.relations, cfg.synthetic_val_relations, cfg.synthetic_test_relations,
                                             args.instances, cfg.max_length, args.vocab, dim, seed=seed)
            splits = [va, te]
            if args.test_file:
                splits.append(FewRelDataset.from_fewrel_json_with_vocab(args.test_file, te.word2id, te.word_vec_mat,
                                                                        cfg.max_length))
            if args.nota_rates:
                for split in splits[1:]:
                    for K in (int(x) for x in args.shots.split(",")):
                        for rate in (float(x) for x in args.nota_rates.split(",")):
                            r = dict(control="meanpool-nearest-prototype", task="transfer", split=split.name, dim=dim,
                                     N=5, K=K, nota_rate=rate, episodes=args.episodes,
                                     **_meanpool_nota(va, split, split.word_vec_mat, K, args.episodes, cfg.seed, rate))
                            rows.append(r)
                            print(json.dumps(r), flush=True)
            for split in splits:
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
