"""FewRel 2.0-style evaluation: NOTA report / threshold selection, domain-adaptation eval, CLI."""
import json
import os
import subprocess
import sys

import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data import make_synthetic
from induction_network_on_fewrel_amd.runtime.evaluate import evaluate_dataset, report, select_nota_threshold

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_report_and_threshold():
    N = 3
    # two episodes x 4 queries; the last query of each is NOTA (label N) with low scores
    probs = torch.tensor([[[0.9, 0.1, 0.1], [0.2, 0.8, 0.1], [0.1, 0.2, 0.7], [0.3, 0.2, 0.25]],
                          [[0.6, 0.1, 0.1], [0.1, 0.1, 0.9], [0.1, 0.7, 0.1], [0.2, 0.35, 0.1]]])
    labels = torch.tensor([[0, 1, 2, 3], [0, 2, 1, 3]])
    r = report(probs, labels, N, 1, 1, 0.25, None)
    assert r.accuracy == 0.75 and r.in_class_accuracy == 1.0 and r.nota_recall == 0.0
    t = select_nota_threshold(probs, labels, N)
    assert 0.35 < t <= 0.6
    r2 = report(probs, labels, N, 1, 1, 0.25, t)
    assert r2.accuracy == 1.0 and r2.nota_precision == 1.0 and r2.nota_recall == 1.0


def test_nota_and_domain_eval_cpu(tmp_path):
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    src = make_synthetic(num_relations=10, instances_per_relation=30, vocab=400, seed=0)
    other = make_synthetic(num_relations=8, instances_per_relation=30, vocab=400, seed=7)   # "another domain"
    other.word_vec_mat = src.word_vec_mat
    cfg = Config(N=5, K=2, Q=3, episodes_per_step=4, model_dir=str(tmp_path / "m"), seed=2, resume=False,
                 nota_rate=0.3, relation_head="paper")
    tr = Trainer(cfg, src, None, device="cpu", log=False, test_data=other)
    for _ in range(2):
        tr.train_step()
    rep = evaluate_dataset(tr, other, 12, 5, 2, 3, nota_rate=0.3, batch=4, tune_iters=8)
    assert rep.episodes == 12 and rep.threshold is not None and 0 < rep.nota_fraction < 1
    assert 0.0 <= rep.accuracy <= 1.0
    # N-independent head: a different way-count at eval time
    rep3 = evaluate_dataset(tr, other, 4, 3, 1, 2, nota_rate=0.0, batch=2)
    assert rep3.N == 3 and rep3.threshold is None


def test_fewrel_eval_cli(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    md = str(tmp_path / "ck")
    common = ["--synthetic", "true", "--synthetic_relations", "8", "--synthetic_instances", "20",
              "--synthetic_vocab", "300", "--device", "cpu", "--model_dir", md, "--relation_head", "paper"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "induction", "5", "1", "--train_iter", "4",
                        "--val_step", "2", "--val_iter", "2", "--test_iter", "2", *common],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([sys.executable, os.path.join(ROOT, "fewrel_eval.py"), "--settings", "5-1,3-2",
                        "--nota_rates", "0,0.5", "--iters", "6", *common],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.strip().splitlines()]
    assert len(rows) == 4 and {(x["N"], x["K"], x["nota_rate"]) for x in rows} == {
        (5, 1, 0.0), (5, 1, 0.5), (3, 2, 0.0), (3, 2, 0.5)}
    assert all(x["step"] >= 2 for x in rows)
