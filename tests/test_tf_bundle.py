"""TF V2 checkpoint bundle written without TF (runtime/tf_bundle.py, the files tf.train.Saver writes for the
reference, model/base.py:124,173-177): byte-level format invariants and round trips.  Parity with a real
TensorFlow reader is unpinned (TF is not installed and the reference ships no checkpoint)."""
import json
import os
import struct
import subprocess
import sys
from collections import OrderedDict

import pytest
import torch

from induction_network_on_fewrel_amd.runtime import checkpoint as ckpt
from induction_network_on_fewrel_amd.runtime import tf_bundle as tb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tensors():
    g = torch.Generator().manual_seed(0)
    return OrderedDict([
        ("bidirectional_rnn/fw/basic_lstm_cell/kernel", torch.randn(35, 80, generator=g)),
        ("bidirectional_rnn/fw/basic_lstm_cell/bias", torch.randn(80, generator=g)),
        ("M", torch.randn(40, 40, 100, generator=g)),
        ("M/Adam", torch.randn(40, 40, 100, generator=g)),
        ("beta1_power", torch.tensor(0.9 ** 3, dtype=torch.float32)),
        ("global_step", torch.tensor(1234, dtype=torch.int64)),
        ("empty", torch.zeros(0, 5)),
        ("ids", torch.arange(7, dtype=torch.int32)),
    ])


def test_crc32c_known_answers():
    assert tb.crc32c(b"123456789") == 0xE3069283            # the CRC-32C check value
    assert tb.crc32c(b"") == 0
    assert tb.crc32c(b"6789", tb.crc32c(b"12345")) == 0xE3069283   # continuation
    from induction_network_on_fewrel_amd.runtime.metrics import crc32c as py_crc
    data = bytes(range(256)) * 17 + b"xyz"
    assert tb.crc32c(data) == py_crc(data)
    for c in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert tb.unmask(tb.mask(c)) == c


def test_header_and_entry_protos():
    # BundleHeaderProto{num_shards: 1, version {producer: 1}} (proto3: LITTLE = 0 is not serialized)
    assert tb.header_proto() == bytes([0x08, 0x01, 0x1A, 0x02, 0x08, 0x01])
    e = tb.entry_proto(1, [40, 100], 300, 16000, 0x12345678)
    assert tb.parse_entry(e) == dict(dtype=1, shape=[40, 100], shard_id=0, offset=300, size=16000, crc32c=0x12345678)
    scalar = tb.entry_proto(9, [], 0, 8, 7)
    assert scalar[:4] == bytes([0x08, 0x09, 0x12, 0x00])   # DT_INT64, empty TensorShapeProto (set, no dims)


def test_empty_block_bytes():
    # LevelDB BlockBuilder::Finish on no entries: one restart point at 0, count 1
    assert tb._block([]) == struct.pack("<II", 0, 1)


def test_bundle_roundtrip_and_format(tmp_path):
    prefix = str(tmp_path / "inductionNetwork-1234")
    t = _tensors()
    tb.save_bundle(prefix, t)
    raw = open(prefix + ".index", "rb").read()
    # footer: two block handles padded to 40 bytes, then the table magic
    assert struct.unpack_from("<Q", raw, len(raw) - 8)[0] == 0xDB4775248B80FB57
    table = tb.read_table(prefix + ".index")       # verifies every block CRC
    keys = list(table)
    assert keys[0] == b"" and keys == sorted(keys) and len(keys) == len(t) + 1
    data = open(prefix + tb.DATA_SUFFIX, "rb").read()
    off = 0
    for k in sorted(t):                              # data in key order, back to back, no padding
        e = tb.parse_entry(table[k.encode()])
        b = t[k].reshape(-1).view(torch.uint8).numpy().tobytes() if t[k].numel() else b""
        assert e["offset"] == off and e["size"] == len(b) and data[off:off + len(b)] == b
        assert tb.unmask(e["crc32c"]) == tb.crc32c(b) and e["shape"] == list(t[k].shape)
        off += len(b)
    assert off == len(data)
    back = tb.load_bundle(prefix)
    for k, v in t.items():
        assert back[k].dtype == v.dtype and torch.equal(back[k], v), k


def test_corruption_is_detected(tmp_path):
    prefix = str(tmp_path / "x-1")
    tb.save_bundle(prefix, _tensors())
    d = bytearray(open(prefix + tb.DATA_SUFFIX, "rb").read())
    d[100] ^= 0x40
    open(prefix + tb.DATA_SUFFIX, "wb").write(bytes(d))
    with pytest.raises(ValueError, match="CRC"):
        tb.load_bundle(prefix)
    i = bytearray(open(prefix + ".index", "rb").read())
    i[5] ^= 0x01
    open(prefix + ".index", "wb").write(bytes(i))
    with pytest.raises(ValueError):
        tb.read_table(prefix + ".index")


def test_many_keys_span_blocks_and_restarts(tmp_path, monkeypatch):
    monkeypatch.setattr(tb, "BLOCK_SIZE", 600)       # several data blocks + index entries
    t = OrderedDict((f"layer_{i:03d}/kernel", torch.full((3,), float(i))) for i in range(70))
    prefix = str(tmp_path / "many-5")
    tb.save_bundle(prefix, t)
    raw = open(prefix + ".index", "rb").read()
    foot = raw[-48:]
    _, i = tb._get_varint(foot, 0)
    _, i = tb._get_varint(foot, i)
    io, i = tb._get_varint(foot, i)
    n, _ = tb._get_varint(foot, i)
    assert len(tb._read_block(raw, io, n)) > 2      # more than two data blocks
    back = tb.load_bundle(prefix)
    assert all(torch.equal(back[k], v) for k, v in t.items())


def test_checkpoint_writes_and_reads_both_formats(tmp_path):
    md = str(tmp_path / "m")
    t = _tensors()
    stem = ckpt.save(md, "inductionNetwork", 1234, t, {"best_acc": 0.5})
    a, ma = ckpt.load(stem)
    b, mb = ckpt.load(stem, prefer="tf")
    for k in t:
        assert torch.equal(a[k], b[k]) and torch.equal(b[k], t[k])
    assert ma == mb and ma["best_acc"] == 0.5
    # a bare TF bundle (no safetensors, no JSON index) still loads
    os.remove(stem + ".safetensors")
    os.remove(stem + ".index.json")
    assert ckpt.latest(md) == stem
    c, mc = ckpt.load(stem)
    assert mc == {"format": "tf-bundle", "global_step": 1234} and torch.equal(c["M"], t["M"])


def test_fewrel_eval_reads_tf_bundle_only_checkpoint(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    md = str(tmp_path / "ck")
    common = ["--synthetic", "true", "--synthetic_relations", "8", "--synthetic_instances", "20",
              "--synthetic_vocab", "300", "--device", "cpu", "--model_dir", md, "--relation_head", "paper"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "induction", "5", "1", "--train_iter", "4",
                        "--val_step", "2", "--val_iter", "2", "--test_iter", "2", *common],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    outs = []
    for fmt in ("safetensors", "tf"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "fewrel_eval.py"), "--settings", "5-1", "--iters", "6",
                            "--checkpoint_format", fmt, "--seed", "3", *common],
                           cwd=tmp_path, capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[0]["accuracy"] == outs[1]["accuracy"] and outs[0]["step"] == outs[1]["step"]


def test_meta_graph_written_and_parsed(tmp_path):
    """<stem>.meta (tf.train.Saver.save writes it next to .index / .data, reference model/base.py:124,177):
    a MetaGraphDef with the model GraphDef + Saver nodes, a V2 SaverDef and the variable collections."""
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.runtime.tb_graph import parse_meta_graph
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    cfg = Config(N=5, K=1, Q=2, hidden_size=8, max_length=12, train_iter=1, val_iter=1, val_step=1000,
                 model_dir=str(tmp_path / "m"), resume=False, device="cpu", dtype="fp32")
    data = make_synthetic(num_relations=8, instances_per_relation=10, vocab=100, seed=0, max_length=12)
    tr = Trainer(cfg, data, None, device="cpu")
    stem = tr.save()
    with open(stem + ".meta", "rb") as fh:
        mg = parse_meta_graph(fh.read())
    assert b"v0" in mg["meta_info"]
    names = {n["name"] for n in mg["nodes"]}
    assert {"save/Const", "save/SaveV2", "save/control_dependency", "save/RestoreV2", "save/restore_all", "M",
            "global_step"} <= names
    sv = mg["saver"]
    assert sv[1] == b"save/Const:0" and sv[2] == b"save/control_dependency:0" and sv[3] == b"save/restore_all"
    assert sv[4] == cfg.max_to_keep and sv[7] == 2 and abs(sv[6] - 10000.0) < 1e-3
    kind, vals = mg["collections"]["trainable_variables"]
    assert kind == 2 and any(v.startswith(b"\n\x03M:0") for v in vals)
    kind, vals = mg["collections"]["variables"]
    assert len(vals) == len(tr.model.params.names()) + 1
    assert mg["collections"]["train_op"] == (1, [b"OptimizeLoss/Adam"])
    # tf_checkpoint=False writes neither the bundle nor the .meta
    cfg2 = Config(**dict(cfg.to_dict(), tf_checkpoint=False, model_dir=str(tmp_path / "n")))
    tr2 = Trainer(cfg2, data, None, device="cpu")
    s2 = tr2.save()
    assert os.path.exists(s2 + ".safetensors") and not os.path.exists(s2 + ".meta") and not os.path.exists(s2 + ".index")


def test_meta_rotated_out_with_its_checkpoint(tmp_path):
    """checkpoint._remove drops a rotated-out stem's .meta with its .index / .data / .safetensors (max_to_keep)."""
    from collections import OrderedDict
    from induction_network_on_fewrel_amd.runtime import checkpoint as ckpt
    md = str(tmp_path / "m")
    t = OrderedDict(w=torch.arange(6, dtype=torch.float32))
    stems = [ckpt.save(md, "inductionNetwork", s, t, {"step": s}, max_to_keep=2, tf_format=True, meta_graph=b"\x0a\x00")
             for s in range(1, 5)]
    for st in stems[:2]:   # rotated out
        assert not any(os.path.exists(st + ext) for ext in (".meta", ".index", ".data-00000-of-00001", ".safetensors"))
    for st in stems[2:]:   # kept
        assert all(os.path.exists(st + ext) for ext in (".meta", ".index", ".safetensors"))
