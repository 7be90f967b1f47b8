"""BERT encoder (north-star addition): tokenisation contract, HF naming, oracle math, trainer plumbing."""
import math

import numpy as np
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data import make_synthetic
from induction_network_on_fewrel_amd.data.bert_tokenize import (BertVocab, encode_instance, features_from_fewrel,
                                                                 synthetic_features)
from induction_network_on_fewrel_amd.models import InductionNetwork
from induction_network_on_fewrel_amd.models import bert as B

TINY = dict(encoder="bert", bert_layers=2, bert_hidden=256, bert_heads=4, bert_intermediate=512, bert_vocab=600,
            bert_max_position=64, bert_max_length=32, bert_out_dim=64)


def test_wordpiece_and_markers():
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]", "[unused0]", "[unused1]", "[unused2]", "[unused3]",
            "the", "cat", "play", "##ing", "##s", "sat"]
    vocab = BertVocab(toks, wordpiece=True)
    assert vocab.marker_ids == [5, 6, 7, 8]            # markers reuse [unused0..3]
    assert vocab.encode_word("Playing") == [11, 12]
    assert vocab.encode_word("plays") == [11, 13]
    assert vocab.encode_word("dog") == [vocab.unk]
    seq, e1, e2 = encode_instance(["The", "cat", "sat"], [1], [2], vocab, 16)
    assert seq == [vocab.cls, 9, 5, 10, 6, 7, 14, 8, vocab.sep]
    assert (e1, e2) == (2, 5) and seq[e1] == 5 and seq[e2] == 7


def test_features_from_fewrel_json_layout():
    ori = {"P1": [{"tokens": ["a", "b", "c", "d"], "h": ["a", "Q1", [[0]]], "t": ["c d", "Q2", [[2, 3]]]}],
           "P2": [{"tokens": ["x"] * 40, "h": ["x", "Q3", [[38]]], "t": ["x", "Q4", [[1]]]}]}
    vocab = BertVocab.from_token_lists(ins["tokens"] for items in ori.values() for ins in items)
    f = features_from_fewrel(ori, vocab, 16)
    assert f["ids"].shape == (2, 16) and f["mask"][0].sum() == f["length"][0]
    # [CLS] [E1] a [/E1] b [E2] c d [/E2] [SEP]
    assert f["length"][0] == 10 and f["e1"][0] == 1 and f["e2"][0] == 5
    assert f["ids"][1, 15] == vocab.sep and f["mask"][1].sum() == 16     # truncated, keeps [SEP]
    assert f["e1"][1] == 15                                             # marker past the cut -> clamped


def test_hf_names_and_counts():
    cfg = Config(**TINY)
    m = InductionNetwork(cfg, None, vocab_size=10)
    names = list(m.params.names().values())
    assert names[0] == "bert.embeddings.word_embeddings.weight"
    assert "bert.encoder.layer.1.attention.self.query.weight" in names
    st = m.params.tf_state()
    assert tuple(st["bert.encoder.layer.0.intermediate.dense.weight"].shape) == (512, 256)   # HF Linear [out, in]
    assert tuple(st["M"].shape) == (64, 64, 100) and tuple(st["bert_proj/kernel"].shape) == (512, 64)
    # q,k,v weights adjacent in the flat order (one [3Hd, Hd] QKV view on the GPU path)
    i = names.index("bert.encoder.layer.0.attention.self.query.weight")
    assert names[i + 1].endswith("key.weight") and names[i + 2].endswith("value.weight")
    full = Config(encoder="bert")
    n = sum(int(np.prod(s)) for s, _ in B.param_specs(full).values())
    bert_base = n - (2 * 768 * 64 + 64)
    assert bert_base == 109_482_240 - (768 * 768 + 768)   # BERT-base (vocab 30522) minus its unused pooler


def test_oracle_layers_match_torch():
    x = torch.randn(3, 7, 16)
    g, b = torch.rand(16) + 0.5, torch.randn(16)
    ref = torch.nn.functional.layer_norm(x, (16,), g, b, eps=1e-12)
    assert torch.allclose(B.layer_norm(x, g, b), ref, atol=1e-5)
    assert torch.allclose(B.gelu(x), torch.nn.functional.gelu(x), atol=1e-6)
    q, k, v = torch.randn(3, 3, 7, 128).unbind(0)
    mask = torch.ones(3, 7, dtype=torch.int32)
    mask[1, 4:] = 0
    out = B.attention(q, k, v, mask, 2, 0, 17, 0.0, False)
    qh, kh, vh = (t.view(3, 7, 2, 64).transpose(1, 2) for t in (q, k, v))
    am = torch.zeros(3, 1, 1, 7).masked_fill(mask[:, None, None, :] == 0, float("-inf"))
    ref = torch.nn.functional.scaled_dot_product_attention(qh, kh, vh, attn_mask=am)
    assert torch.allclose(out, ref.transpose(1, 2).reshape(3, 7, 128), atol=1e-5)


def test_dropout_mask_rate():
    m = B.keep_mask(3, 17, 100000, 0.9)
    assert abs(float(m.mean()) - 0.9) < 0.005
    assert torch.equal(m, B.keep_mask(3, 17, 100000, 0.9)) and not torch.equal(m, B.keep_mask(3, 18, 100000, 0.9))


def test_bert_model_trains_cpu(tmp_path):
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=8, instances_per_relation=20, max_length=20, vocab=500, seed=0)
    cfg = Config(N=5, K=2, Q=2, episodes_per_step=2, model_dir=str(tmp_path / "m"), seed=1, resume=False,
                 learning_rate=1e-3, lr_schedule="constant", **TINY)
    tr = Trainer(cfg, data, None, device="cpu", log=False)
    assert tr.train_data.bert is not None and tr.train_data.bert["ids"].shape == (160, 32)
    before = tr.flat.flat.clone()
    losses = [tr.train_step()[0] for _ in range(3)]
    assert all(math.isfinite(x) for x in losses)
    assert not torch.equal(before, tr.flat.flat)
    # every parameter group received a gradient at some point
    g = tr.flat.grad
    assert float(g.abs().sum()) > 0
    acc = tr.evaluate(4)
    assert 0.0 <= acc <= 1.0
    tr.save()
    tr2 = Trainer(cfg.replace(resume=True), data, None, device="cpu", log=False)
    assert tr2.global_step == 3 and torch.equal(tr2.flat.flat, tr.flat.flat)


def test_synthetic_features_markers():
    data = make_synthetic(num_relations=2, instances_per_relation=3, max_length=12, vocab=50, seed=0)
    f = synthetic_features(data, 100, 20)
    for i in range(6):
        assert f["ids"][i, 0] == 2 and f["ids"][i, f["length"][i] - 1] == 3
        assert f["ids"][i, f["e1"][i]] == 5 and f["ids"][i, f["e2"][i]] == 7
        assert f["ids"][i].max() < 100


def _tiny_hf(tmp_path, fmt="safetensors", prefix=False):
    """A random transformers.BertModel built offline from a tiny BertConfig, saved to a local dir."""
    import os
    import transformers
    hc = transformers.BertConfig(vocab_size=600, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                 intermediate_size=512, max_position_embeddings=64, hidden_dropout_prob=0.0,
                                 attention_probs_dropout_prob=0.0, hidden_act="gelu", layer_norm_eps=1e-12)
    torch.manual_seed(11)
    hf = transformers.BertModel(hc, add_pooling_layer=True).eval()
    with torch.no_grad():   # non-trivial LayerNorm affine / biases
        for n, t in hf.named_parameters():
            if "LayerNorm" in n or n.endswith("bias"):
                t.add_(torch.randn_like(t) * 0.1)
    d = str(tmp_path / f"hf_{fmt}_{int(prefix)}")
    if fmt == "safetensors":
        hf.save_pretrained(d, safe_serialization=True)
    else:
        os.makedirs(d, exist_ok=True)
        sd = {("bert." + k if prefix else k): v.clone() for k, v in hf.state_dict().items()}
        torch.save(sd, os.path.join(d, "pytorch_model.bin"))
    return hf, d


def _hidden_vs_hf(hf, d):
    cfg = Config(**dict(TINY, bert_checkpoint=d, bert_dropout=0.0, bert_attn_dropout=0.0))
    m = InductionNetwork(cfg, None, vocab_size=10, seed=0)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 600, (3, 32), generator=g)
    mask = torch.ones(3, 32, dtype=torch.int64)
    mask[1, 20:] = 0
    mask[2, 7:] = 0
    with torch.no_grad():
        ours = B.hidden_states_ref(m.bert_pdict(), ids, mask, cfg)
        ref_h = hf(input_ids=ids, attention_mask=mask).last_hidden_state
    valid = mask.bool()
    return float((ours - ref_h)[valid].abs().max()), float(ref_h[valid].abs().max())


def test_bert_checkpoint_matches_hf_bertmodel(tmp_path):
    """bert_checkpoint: a saved transformers.BertModel (model.safetensors) loads by name, and our
    oracle encoder reproduces its last_hidden_state (dropout 0) -- the HF-layout claim, pinned."""
    hf, d = _tiny_hf(tmp_path, "safetensors")
    err, mx = _hidden_vs_hf(hf, d)
    assert err < 2e-5 * max(1.0, mx), err


def test_bert_checkpoint_torch_bin_with_prefix(tmp_path):
    """pytorch_model.bin (weights_only load) with task-model ``bert.`` keys and a pooler to ignore."""
    hf, d = _tiny_hf(tmp_path, "bin", prefix=True)
    err, mx = _hidden_vs_hf(hf, d)
    assert err < 2e-5 * max(1.0, mx), err


def test_bert_checkpoint_shape_mismatch_is_loud(tmp_path):
    import pytest
    hf, d = _tiny_hf(tmp_path, "safetensors")
    with pytest.raises(ValueError, match="shape"):
        InductionNetwork(Config(**dict(TINY, bert_checkpoint=d, bert_intermediate=1024)), None, vocab_size=10)
