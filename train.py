#!/usr/bin/env python3
"""Train / evaluate the Induction Network (CLI-compatible with the reference ``train.py``).

Reference: ``python train.py [model_name=induction] [N=5] [K=2]`` with Q=5, max_length=37,
hidden_size=20, ``./data/glove.6B.5d.json`` and ``checkpoints/inductionNetwork_test``
(train.py:10-39). The same positional form works here; every Config field is also a ``--flag``.

Examples
  python train.py induction 5 2                          # reference defaults (needs data files)
  python train.py induction 5 1 --synthetic true         # synthetic FewRel-shaped data
  python train.py induction 5 1 --synthetic true --synthetic_task transfer --test_best true   # unseen relations
  python train.py induction 5 5 --val_file data/val.json --split_val true   # relation-disjoint val split
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py induction 5 5 --episodes_per_step 64
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from induction_network_on_fewrel_amd.config import Config, add_cli_args, config_from_args  # noqa: E402


def build_parser():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("pos_model_name", nargs="?", default=None)
    p.add_argument("pos_N", nargs="?", type=int, default=None)
    p.add_argument("pos_K", nargs="?", type=int, default=None)
    add_cli_args(p)
    p.add_argument("--split_val", type=lambda s: s.lower() in ("1", "true", "yes"), default=False,
                   help="train.json is absent: split val.json's relations into disjoint train/val halves")
    p.add_argument("--eval_only", type=lambda s: s.lower() in ("1", "true", "yes"), default=False)
    p.add_argument("--train_relations", type=int, default=0,
                   help="with --split_val: how many of val.json's relations train (default: half)")
    p.add_argument("--fold", type=int, default=-1,
                   help="with --split_val (relation mode): hold out relations 5*fold .. 5*fold+4 (JSON order, "
                        "wrapping) and train on the rest -- rotating folds for mean +- std accuracy")
    p.add_argument("--val_relations", type=int, default=0,
                   help="with --fold: a THIRD relation-disjoint block -- the V relations after the held-out test "
                        "block (JSON order, wrapping) are the validation set that selects the checkpoint "
                        "(--test_best), the fold's 5 relations are only tested, the rest train")
    p.add_argument("--split_mode", default="relation", choices=["relation", "instance"],
                   help="with --split_val: 'relation' = disjoint relations (few-shot transfer); 'instance' = "
                        "every relation in both halves, disjoint sentences (train_fraction of each relation)")
    p.add_argument("--train_fraction", type=float, default=0.7,
                   help="with --split_mode instance: leading fraction of each relation's instances that trains")
    p.add_argument("--vocab_from_data", type=lambda s: s.lower() in ("1", "true", "yes"), default=False,
                   help="no GloVe file: build a random word table from the data's tokens")
    return p


def load_data(cfg: Config, args):
    from induction_network_on_fewrel_amd.data import FewRelDataset, make_synthetic, vocab_from_fewrel
    if cfg.synthetic and cfg.synthetic_task == "transfer":   # relation-disjoint train / val / test
        from induction_network_on_fewrel_amd.data.synthetic import make_transfer_splits
        tr, va, te = make_transfer_splits(cfg.synthetic_relations, cfg.synthetic_val_relations,
                                          cfg.synthetic_test_relations, cfg.synthetic_instances, cfg.max_length,
                                          cfg.synthetic_vocab, cfg.synthetic_word_dim, seed=cfg.seed)
        print(f"transfer task: {len(tr.relations())} train / {len(va.relations())} val / {len(te.relations())} test "
              "relations (disjoint trigger tokens)", flush=True)
        args._test_split = te
        return tr, va
    if cfg.synthetic:
        tr = make_synthetic(cfg.synthetic_relations, cfg.synthetic_instances, cfg.max_length, cfg.synthetic_vocab,
                            cfg.synthetic_word_dim, seed=cfg.seed)
        va = make_synthetic(max(cfg.N + 1, 16), cfg.synthetic_instances, cfg.max_length, cfg.synthetic_vocab,
                            cfg.synthetic_word_dim, seed=cfg.seed + 1)
        va.word_vec_mat = tr.word_vec_mat
        return tr, va
    wv = cfg.word_vec_file
    if args.vocab_from_data or not os.path.exists(wv):
        src = cfg.val_file if args.split_val or not os.path.exists(cfg.train_file) else cfg.train_file
        wv = os.path.join(cfg.processed_dir, "vocab_from_data.json")
        if not os.path.exists(wv):
            os.makedirs(cfg.processed_dir, exist_ok=True)
            with open(wv, "w") as fh:
                json.dump(vocab_from_fewrel(src, dim=cfg.synthetic_word_dim, seed=cfg.seed), fh)
    if args.split_val or not os.path.exists(cfg.train_file):
        full = FewRelDataset.from_json(cfg.val_file, wv, cfg.max_length, cfg.case_sensitive,
                                       processed_dir=cfg.processed_dir)
        rels = full.relations()
        if getattr(args, "split_mode", "relation") == "instance":
            f = args.train_fraction
            if cfg.encoder == "bert":
                raise SystemExit("--split_mode instance is implemented for the BiLSTM encoder")
            return (full.subset_relations(rels, "train_split", part=(0.0, f)),
                    full.subset_relations(rels, "val_split", part=(f, 1.0)))
        if getattr(args, "fold", -1) >= 0:   # rotate: the held-out block of 5 relations goes last
            test = [rels[(5 * args.fold + i) % len(rels)] for i in range(5)]
            nv = getattr(args, "val_relations", 0)
            if nv > 0:   # train / val / test, all relation-disjoint: val selects, test only tests
                if cfg.encoder == "bert":
                    raise SystemExit("--val_relations is implemented for the BiLSTM encoder")
                # the val block must not wrap into the test block, and N relations must remain for training
                if 5 + nv > len(rels) - cfg.N:
                    raise SystemExit(f"--val_relations {nv}: {len(rels)} relations leave no disjoint train / val / "
                                     f"test split with >= {cfg.N} training relations (need 5 + val <= {len(rels) - cfg.N})")
                val = [rels[(5 * args.fold + 5 + i) % len(rels)] for i in range(nv)]
                assert not set(val) & set(test)
                train = [r for r in rels if r not in test and r not in val]
                print(f"fold {args.fold}: train {len(train)} relations, val {val}, test {test}", flush=True)
                args._test_split = full.subset_relations(test, "test_split")
                return full.subset_relations(train, "train_split"), full.subset_relations(val, "val_split")
            rels = [r for r in rels if r not in test] + test
            half = len(rels) - 5
            print(f"fold {args.fold}: held-out relations {test}", flush=True)
        else:
            half = args.train_relations or len(rels) // 2
        tr, va = full.subset_relations(rels[:half], "train_split"), full.subset_relations(rels[half:], "val_split")
        return _with_bert(cfg, tr, va, cfg.val_file, full, rels, half)
    tr = FewRelDataset.from_json(cfg.train_file, wv, cfg.max_length, cfg.case_sensitive, processed_dir=cfg.processed_dir)
    va = FewRelDataset.from_json(cfg.val_file, wv, cfg.max_length, cfg.case_sensitive, processed_dir=cfg.processed_dir)
    if cfg.encoder == "bert":
        from induction_network_on_fewrel_amd.data.bert_tokenize import features_from_json
        tr.bert, vocab = features_from_json(cfg.train_file, cfg.bert_max_length, vocab_file=cfg.bert_vocab_file)
        va.bert, _ = features_from_json(cfg.val_file, cfg.bert_max_length, vocab=vocab)
    return tr, va


def load_test(cfg: Config, tr):
    """A separate test file (e.g. another domain, FewRel 2.0 DA) tensorised with the training vocabulary."""
    from induction_network_on_fewrel_amd.data import FewRelDataset
    if tr.word2id is None:
        raise SystemExit("--test_file needs a vocabulary-backed training set (not --synthetic)")
    te = FewRelDataset.from_fewrel_json_with_vocab(cfg.test_file, tr.word2id, tr.word_vec_mat, cfg.max_length,
                                                   cfg.case_sensitive)
    if cfg.encoder == "bert":
        from induction_network_on_fewrel_amd.data.bert_tokenize import features_from_json
        te.bert, _ = features_from_json(cfg.test_file, cfg.bert_max_length, vocab=getattr(tr, "bert_vocab", None),
                                        vocab_file=cfg.bert_vocab_file)
    return te


def _with_bert(cfg, tr, va, path, full, rels, half):
    """BERT features for a relation split of one JSON file (same instance order as the split)."""
    if cfg.encoder != "bert":
        return tr, va
    from induction_network_on_fewrel_amd.data.bert_tokenize import features_from_json
    full.bert, _ = features_from_json(path, cfg.bert_max_length, vocab_file=cfg.bert_vocab_file)
    return full.subset_relations(rels[:half], "train_split"), full.subset_relations(rels[half:], "val_split")


def main(argv=None):
    args = build_parser().parse_args(argv)
    cfg = config_from_args(args, Config())
    pos = {}
    if args.pos_model_name is not None:
        pos["model_name"] = args.pos_model_name
    if args.pos_N is not None:
        pos["N"] = args.pos_N
    if args.pos_K is not None:
        pos["K"] = args.pos_K
    cfg = cfg.replace(**pos)
    cfg.validate()
    if cfg.model_name != "induction":
        raise SystemExit(f"unknown model {cfg.model_name!r} (only 'induction')")
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    tr_data, va_data = load_data(cfg, args)
    te_data = load_test(cfg, tr_data) if cfg.test_file else getattr(args, "_test_split", None)
    trainer = Trainer(cfg, tr_data, va_data, device=cfg.device, test_data=te_data)
    if args.eval_only:
        acc = trainer.evaluate(cfg.test_iter)
        if trainer.dist.is_main:
            print(json.dumps({"eval_accuracy": acc, "episodes": cfg.test_iter, "N": cfg.eN, "K": cfg.eK}))
    else:
        trainer.train()
    trainer.dist.destroy()


if __name__ == "__main__":
    main()
