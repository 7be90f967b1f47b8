#!/usr/bin/env python3
"""Evaluate a trained Induction Network checkpoint FewRel-2.0 style (no reference counterpart: the
reference only reports plain accuracy on its val loader, model/base.py:186-208).

  python fewrel_eval.py --model_dir checkpoints/run --val_file data/val.json --N 5 --K 1 \\
      --settings 5-1,5-5,10-1,10-5 --nota_rates 0,0.15,0.5 [--test_file other_domain.json]

* loads the latest checkpoint of ``--model_dir`` (config from the checkpoint's metadata, overridable
  by flags), rebuilds the vocabulary the same way train.py does;
* ``--test_file``: domain-adaptation evaluation (a file from another domain, tensorised with the
  training vocabulary); default is the validation data;
* NOTA thresholds are tuned on the validation data unless ``--nota_threshold`` is given;
* prints one JSON line per (N, K, NOTA rate): accuracy, in-class accuracy, NOTA precision / recall.
Different N than trained requires ``relation_head=paper`` (the reference head's FC is N-specific).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None):
    import train as T
    from induction_network_on_fewrel_amd.config import Config, config_from_args
    from induction_network_on_fewrel_amd.runtime import checkpoint as ckpt
    from induction_network_on_fewrel_amd.runtime.evaluate import evaluate_dataset
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer

    p = T.build_parser()
    p.add_argument("--settings", default="", help="comma list of N-K (default: the config's eval N/K)")
    p.add_argument("--nota_rates", default="0")
    p.add_argument("--iters", type=int, default=1000)
    p.add_argument("--checkpoint", default="best", choices=["best", "latest"],
                   help="best-val checkpoint (falls back to the latest) or the latest one")
    p.add_argument("--checkpoint_format", default="safetensors", choices=["safetensors", "tf"],
                   help="read the safetensors copy or the TF V2 bundle (.index + .data-00000-of-00001); a "
                        "checkpoint with only one of them loads from that one")
    args = p.parse_args(argv)
    base = Config()
    md = args.model_dir or base.model_dir
    stem = (ckpt.best(md) if args.checkpoint == "best" else None) or ckpt.latest(md)
    if stem is not None:
        _, meta = ckpt.load(stem, args.checkpoint_format)
        base = Config.from_dict(meta.get("config", {}))
    cfg = config_from_args(args, base).replace(resume=False, episodes_per_step=max(1, base.episodes_per_step))
    tr_data, va_data = T.load_data(cfg, args)
    # --test_file (another domain) > the task's held-out test relations (synthetic transfer, --fold with
    # --val_relations) > the validation data
    te = T.load_test(cfg, tr_data) if cfg.test_file else (getattr(args, "_test_split", None) or va_data)
    trainer = Trainer(cfg, tr_data, va_data, device=cfg.device, log=False)
    if stem is not None:
        trainer.load(stem, args.checkpoint_format)
    else:
        print(json.dumps({"warning": "no checkpoint found; evaluating the random init"}), file=sys.stderr)
    settings = ([tuple(int(x) for x in s.split("-")) for s in args.settings.split(",") if s]
                or [(cfg.eN, cfg.eK)])
    rates = [float(x) for x in args.nota_rates.split(",")]
    thr = cfg.nota_threshold if cfg.nota_threshold >= 0 else None
    for N, K in settings:
        for r in rates:
            rep = evaluate_dataset(trainer, te, args.iters, N, K, cfg.eQ, r, thr if r > 0 else None,
                                   cfg.eval_batch or None, tune_on=va_data)
            if trainer.dist.is_main:
                print(json.dumps(dict(rep.to_dict(), data=os.path.basename(cfg.test_file) if cfg.test_file
                                      else te.name, head=cfg.relation_head, step=trainer.global_step)))
    trainer.dist.destroy()


if __name__ == "__main__":
    main()
