"""Runtime: optimizer math, LR schedule, checkpoint layout + resume, metrics event files, trainer."""
import math
import os

import numpy as np
import pytest
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data import make_synthetic
from induction_network_on_fewrel_amd.ops.optim import FlatParams, FusedOptimizer, lr_at
from induction_network_on_fewrel_amd.runtime import checkpoint as ckpt
from induction_network_on_fewrel_amd.runtime.metrics import EventWriter, crc32c, read_events


def test_lr_staircase_matches_tf_exponential_decay():
    assert lr_at(0, 1e-3, 100, 0.9) == 1e-3
    assert lr_at(99, 1e-3, 100, 0.9) == 1e-3
    assert abs(lr_at(100, 1e-3, 100, 0.9) - 9e-4) < 1e-12
    assert abs(lr_at(10000, 1e-3, 100, 0.9) - 1e-3 * 0.9 ** 100) < 1e-15   # the reference's LR collapse
    assert abs(lr_at(150, 1e-3, 100, 0.9, staircase=False) - 1e-3 * 0.9 ** 1.5) < 1e-12


def test_fused_adam_cpu_matches_tf1_adam():
    p = torch.nn.Parameter(torch.randn(50))
    flat = FlatParams({"x": p})
    opt = FusedOptimizer(flat, "adam")
    ref_p = p.detach().clone()
    m = torch.zeros(50)
    v = torch.zeros(50)
    for t in range(1, 6):
        g = torch.randn(50)
        flat.grad.copy_(g)
        opt.step(1e-2)
        m = 0.9 * m + 0.1 * g
        v = 0.999 * v + 0.001 * g * g
        lr_t = 1e-2 * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        ref_p = ref_p - lr_t * m / (v.sqrt() + 1e-8)
    assert torch.allclose(p.detach(), ref_p, atol=1e-6)


def test_flat_params_are_views():
    a = torch.nn.Parameter(torch.ones(3, 2))
    b = torch.nn.Parameter(torch.zeros(4))
    flat = FlatParams({"a": a, "b": b})
    flat.flat.fill_(2.0)
    assert float(a.sum()) == 12 and float(b.sum()) == 8
    (a.sum() * 3 + b.sum()).backward()
    flat.sync_grads_into_flat()
    assert torch.allclose(flat.grad, torch.tensor([3.0] * 6 + [1.0] * 4))


def test_checkpoint_layout_and_rotation(tmp_path):
    md = str(tmp_path / "m")
    for step in (10, 20, 30):
        ckpt.save(md, "inductionNetwork", step, {"W_s": torch.ones(2, 2) * step, "global_step": torch.tensor(step)},
                  {"best_acc": step / 100}, max_to_keep=2)
    d = os.path.join(md, "checkpoint")
    files = sorted(os.listdir(d))
    assert files == ["checkpoint",
                     "inductionNetwork-20.data-00000-of-00001", "inductionNetwork-20.index",
                     "inductionNetwork-20.index.json", "inductionNetwork-20.safetensors",
                     "inductionNetwork-30.data-00000-of-00001", "inductionNetwork-30.index",
                     "inductionNetwork-30.index.json", "inductionNetwork-30.safetensors"]
    with open(os.path.join(d, "checkpoint")) as fh:
        txt = fh.read()
    assert 'model_checkpoint_path: "inductionNetwork-30"' in txt
    t, meta = ckpt.load(ckpt.latest(md))
    assert float(t["W_s"][0, 0]) == 30 and meta["best_acc"] == 0.3 and meta["variables"]["W_s"]["shape"] == [2, 2]


def test_best_checkpoint_survives_rotation_and_newer_saves(tmp_path):
    md = str(tmp_path / "m")
    t = lambda step: {"W_s": torch.ones(2, 2) * step, "global_step": torch.tensor(step)}
    ckpt.save(md, "inductionNetwork", 2, t(2), {}, max_to_keep=2, best=True)
    for step in (4, 6, 8):   # periodic checkpoints after the best one
        ckpt.save(md, "inductionNetwork", step, t(step), {}, max_to_keep=2)
    assert ckpt.latest(md).endswith("inductionNetwork-8")
    assert ckpt.best(md).endswith("inductionNetwork-2")
    assert float(ckpt.load(ckpt.best(md))[0]["W_s"][0, 0]) == 2
    files = sorted(os.listdir(os.path.join(md, "checkpoint")))
    assert "inductionNetwork-4.safetensors" not in files and "inductionNetwork-2.safetensors" in files


def test_superseded_best_is_deleted(tmp_path):
    """Advisor finding: a best that left the rotation and is then beaten must not stay on disk."""
    md = str(tmp_path / "m")
    t = lambda step: {"W_s": torch.ones(2, 2) * step, "global_step": torch.tensor(step)}
    ckpt.save(md, "inductionNetwork", 2, t(2), {}, max_to_keep=2, best=True)
    for step in (4, 6, 8):
        ckpt.save(md, "inductionNetwork", step, t(step), {}, max_to_keep=2)
    ckpt.save(md, "inductionNetwork", 10, t(10), {}, max_to_keep=2, best=True)   # beats best-2
    files = sorted(os.listdir(os.path.join(md, "checkpoint")))
    assert "inductionNetwork-2.safetensors" not in files and "inductionNetwork-2.index.json" not in files
    assert ckpt.best(md).endswith("inductionNetwork-10")
    # a best still inside the rotation is left to the rotation (it is a regular checkpoint too)
    ckpt.save(md, "inductionNetwork", 12, t(12), {}, max_to_keep=2, best=True)
    files = sorted(os.listdir(os.path.join(md, "checkpoint")))
    assert "inductionNetwork-10.safetensors" in files and ckpt.best(md).endswith("inductionNetwork-12")
    ckpt.save(md, "inductionNetwork", 14, t(14), {}, max_to_keep=2)
    files = sorted(os.listdir(os.path.join(md, "checkpoint")))
    assert [f for f in files if f.endswith(".safetensors")] == ["inductionNetwork-12.safetensors",
                                                                "inductionNetwork-14.safetensors"]


def test_test_best_loads_best_not_latest(tmp_path):
    """test_best with periodic saves: the final test must run on the best-val weights."""
    tr = _trainer(tmp_path, resume=False, save_every=1, train_iter=4, val_step=2, val_iter=2, test_iter=2,
                  test_best=True, log_every=1)
    accs = iter([0.9, 0.1])   # val at step 2 is the best, val at step 4 is worse
    tr.evaluate = lambda iters, **kw: next(accs, 0.5)
    loaded = []
    orig = tr.load
    tr.load = lambda stem: (loaded.append(stem), orig(stem))
    tr.train()
    assert loaded and loaded[0].endswith("inductionNetwork-2"), loaded


def test_nonfinite_gradient_skips_update_cpu():
    p = torch.nn.Parameter(torch.randn(10))
    flat = FlatParams({"x": p})
    opt = FusedOptimizer(flat, "adam")
    flat.grad.copy_(torch.randn(10))
    opt.step(1e-2, check_finite=True)
    p1, m1, v1 = flat.flat.clone(), opt.m.clone(), opt.v.clone()
    flat.grad[3] = float("nan")
    opt.step(1e-2, check_finite=True)
    assert torch.equal(flat.flat, p1) and torch.equal(opt.m, m1) and torch.equal(opt.v, v1)
    assert opt.skipped() == 1
    flat.grad.fill_(0.5)
    opt.step(1e-2, check_finite=True, loss=torch.tensor(float("inf")))
    assert opt.skipped() == 2 and torch.equal(flat.flat, p1)


def test_event_file_roundtrip(tmp_path):
    assert crc32c(b"123456789") == 0xE3069283   # CRC-32C check value
    w = EventWriter(str(tmp_path))
    w.scalars(1, {"loss": 0.5, "accuracy": 0.25})
    w.scalars(2, {"loss": 0.25})
    w.close()
    ev = read_events(w.path)
    assert ev[1][0] == 1 and abs(ev[1][1]["loss"] - 0.5) < 1e-7 and abs(ev[1][1]["accuracy"] - 0.25) < 1e-7
    assert ev[2] == (2, {"loss": 0.25})


def _trainer(tmp_path, B=4, **kw):
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=10, instances_per_relation=40, vocab=500, seed=0)
    cfg = Config(N=5, K=2, Q=3, episodes_per_step=B, model_dir=str(tmp_path / "run"), seed=3, **kw)
    return Trainer(cfg, data, None, device="cpu", log=False)


def test_checkpoint_resume_is_bitwise(tmp_path):
    tr = _trainer(tmp_path, resume=False)
    for _ in range(3):
        tr.train_step()
    tr.save()
    ref_losses = [tr.train_step()[0] for _ in range(2)]
    ref_params = tr.flat.flat.clone()
    tr2 = _trainer(tmp_path, resume=True)
    assert tr2.global_step == 3
    losses = [tr2.train_step()[0] for _ in range(2)]
    assert losses == ref_losses
    assert torch.equal(tr2.flat.flat, ref_params)
    names = set(ckpt.load(ckpt.latest(str(tmp_path / "run")))[0].keys())
    assert {"M", "M/Adam", "M/Adam_1", "beta1_power", "beta2_power", "global_step", "embedding/Variable"} <= names


@pytest.mark.slow
def test_training_learns_on_synthetic(tmp_path):
    """The model has a long MSE plateau (~0.16) before it separates classes; ~500 episodes-steps of
    8 episodes at lr 1e-2 get it well above chance on the synthetic trigger-token task."""
    tr = _trainer(tmp_path, B=8, resume=False, learning_rate=1e-2, lr_schedule="constant", keep_prob=1.0)
    first = [tr.train_step()[0] for _ in range(5)]
    for _ in range(560):
        tr.train_step()
    last = [tr.train_step()[0] for _ in range(5)]
    acc = tr.evaluate(60)
    assert np.mean(last) < np.mean(first)
    assert acc > 0.3   # chance = 0.2


def test_fault_injection_then_resume(tmp_path):
    """Failure detection / restart: a rank dies mid-run (INA_FAULT_STEP), the relaunch resumes from the
    last periodic checkpoint and finishes."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [sys.executable, os.path.join(root, "train.py"), "induction", "5", "1", "--synthetic", "true",
            "--synthetic_relations", "8", "--synthetic_instances", "20", "--synthetic_vocab", "300",
            "--train_iter", "8", "--val_step", "100", "--val_iter", "2", "--test_iter", "2", "--log_every", "1",
            "--save_every", "2", "--device", "cpu", "--watchdog_s", "600", "--model_dir", str(tmp_path / "ck")]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", INA_FAULT_STEP="5")
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env, cwd=tmp_path)
    assert r.returncode != 0 and "injected fault at step 5" in r.stderr
    env.pop("INA_FAULT_STEP")
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "resumed from" in r.stdout and "inductionNetwork-4" in r.stdout
    assert "Test accuracy" in r.stdout


def test_gradient_norm_summaries(tmp_path):
    """optimize_loss's gradient summaries (model/base.py:98,113): the global norm of the last step's
    gradient and, on request, one norm per TF variable -- in metrics.jsonl and the TensorBoard file."""
    import glob
    import json
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=10, instances_per_relation=40, vocab=500, seed=0)
    cfg = Config(N=5, K=2, Q=3, episodes_per_step=2, model_dir=str(tmp_path / "run"), seed=3, resume=False,
                 train_iter=3, val_step=1000, test_iter=2, log_every=1,
                 summaries="loss,learning_rate,global_gradient_norm,gradient_norm")
    tr = Trainer(cfg, data, None, device="cpu", log=True)
    tr.train_step()
    norms = tr.gradient_norms(per_variable=True)
    g = tr.flat.grad
    assert abs(norms["global_norm/gradient_norm"] - float(g.norm())) < 1e-4 * float(g.norm())
    ms = tr.flat.view(g, "M")
    assert abs(norms["gradient_norm/M"] - float(ms.norm())) < 1e-3 * float(ms.norm())
    assert "gradient_norm/bidirectional_rnn/fw/basic_lstm_cell/kernel" in norms
    tr.train()
    recs = [json.loads(x) for x in open(tmp_path / "run" / "train" / "metrics.jsonl")]
    tr_recs = [r for r in recs if r["kind"] == "train"]
    assert tr_recs and all("global_norm/gradient_norm" in r and "gradient_norm/M" in r for r in tr_recs)
    ev = read_events(glob.glob(str(tmp_path / "run" / "train" / "events.out.tfevents.*"))[0])
    tags = set().union(*(v.keys() for _, v in ev))
    assert {"loss", "learning_rate", "global_norm/gradient_norm", "gradient_norm/M"} <= tags


def test_tensorboard_graph(tmp_path):
    """The model graph event (reference: FileWriter(..., sess.graph), model/base.py:125): the reference's
    placeholders, every variable under its TF name with its shape, and the module scopes."""
    import glob
    from induction_network_on_fewrel_amd.runtime.tb_graph import read_graph
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=10, instances_per_relation=40, vocab=500, seed=0)
    cfg = Config(N=5, K=2, Q=3, episodes_per_step=2, model_dir=str(tmp_path / "run"), seed=3, resume=False,
                 train_iter=1, val_step=1000, test_iter=2, log_every=1)
    tr = Trainer(cfg, data, None, device="cpu", log=True)
    tr.log.flush()
    nodes = read_graph(glob.glob(str(tmp_path / "run" / "train" / "events.out.tfevents.*"))[0])
    by = {n["name"]: n for n in nodes}
    for ph in ("input_words", "input_pos1", "input_pos2", "mask_padding", "query_label", "keep_probx"):
        assert by[ph]["op"] == "Placeholder", ph
    for attr, name in tr.model.params.names().items():
        assert by[name]["op"] == "VariableV2" and by[name + "/read"]["inputs"] == [name], name
        assert "shape" in by[name]["attrs"]
    scopes = {n["name"].split("/")[0] for n in nodes}
    assert {"embedding", "EncoderModule", "InductionModule", "RelationModule", "loss"} <= scopes
    names = set(by)
    for n in nodes:   # every input is a node of the graph
        assert all(i in names for i in n["inputs"]), n["name"]


def test_legacy_single_sampler_checkpoint_resumes_exactly(tmp_path):
    """Advisor finding: an older checkpoint with one 'train_sampler' entry must restore the CPU
    sampler's RNG in full at world size 1 (not restart it and replay episodes)."""
    import json
    tr = _trainer(tmp_path, resume=False)
    tr.train_step()
    stem = tr.save()
    cont = tr.train_eps.sample(4, 5, 2, 3)[0]
    idx = stem + ".index.json"
    meta = json.load(open(idx))
    meta["train_sampler"] = meta.pop("train_samplers")[0]   # the pre-DP checkpoint format
    json.dump(meta, open(idx, "w"))
    tr2 = _trainer(tmp_path, resume=True)
    assert torch.equal(tr2.train_eps.sample(4, 5, 2, 3)[0], cont)
