"""train.py keeps the reference CLI (``train.py [model_name] [N] [K]``) and runs end to end on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAL = "/root/reference/data/val.json"


def _run(args, cwd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    return subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), *args], cwd=cwd, capture_output=True,
                          text=True, timeout=600, env=env)


def test_positional_cli_synthetic(tmp_path):
    r = _run(["induction", "5", "1", "--synthetic", "true", "--synthetic_relations", "8",
              "--synthetic_instances", "20", "--synthetic_vocab", "300", "--train_iter", "4", "--val_step", "2",
              "--val_iter", "2", "--test_iter", "2", "--log_every", "2", "--device", "cpu",
              "--model_dir", str(tmp_path / "ck")], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "5-way-1-shot Few-Shot Relation Classification" in r.stdout
    assert "Test accuracy:" in r.stdout
    assert os.path.exists(tmp_path / "ck" / "checkpoint" / "checkpoint")
    assert (tmp_path / "ck" / "train" / "metrics.jsonl").exists()
    recs = [json.loads(x) for x in open(tmp_path / "ck" / "train" / "metrics.jsonl")]
    assert {r["kind"] for r in recs} >= {"train", "val", "test"}


@pytest.mark.skipif(not os.path.exists(VAL), reason="reference val.json not mounted")
def test_real_val_json_relation_split(tmp_path):
    r = _run(["induction", "5", "2", "--val_file", VAL, "--split_val", "true", "--vocab_from_data", "true",
              "--processed_dir", str(tmp_path / "_processed_data"), "--train_iter", "2", "--val_step", "2",
              "--val_iter", "2", "--test_iter", "2", "--device", "cpu", "--model_dir", str(tmp_path / "ck")], tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Test accuracy:" in r.stdout


@pytest.mark.skipif(not os.path.exists(VAL), reason="reference val.json not mounted")
def test_val_relations_must_not_reach_the_test_block(tmp_path):
    """--fold with --val_relations: the validation block may not wrap into the held-out test relations."""
    r = _run(["induction", "5", "1", "--val_file", VAL, "--split_val", "true", "--vocab_from_data", "true",
              "--processed_dir", str(tmp_path / "_processed_data"), "--fold", "0", "--val_relations", "9",
              "--train_iter", "2", "--device", "cpu", "--model_dir", str(tmp_path / "ck")], tmp_path)
    assert r.returncode != 0 and "no disjoint train / val / test split" in (r.stderr + r.stdout)


def test_deterministic_cpu_train_steps_repeat(tmp_path):
    """Config.deterministic (torch deterministic algorithms, errors rather than warnings): two CPU runs of the
    same seed give bitwise-equal parameters."""
    import torch
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data.synthetic import make_synthetic
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=8, instances_per_relation=20, vocab=300, seed=0)
    flats = []
    try:
        for i in range(2):
            cfg = Config(N=5, K=1, Q=2, episodes_per_step=2, model_dir=str(tmp_path / f"d{i}"), seed=3, resume=False,
                         deterministic=True, device="cpu")
            tr = Trainer(cfg, data, None, device="cpu", log=False)
            for _ in range(2):
                tr.train_step()
            flats.append(tr.flat.flat.detach().clone())
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.equal(flats[0], flats[1])
