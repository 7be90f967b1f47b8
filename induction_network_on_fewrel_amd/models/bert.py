"""BERT sentence encoder for the Induction Network (north-star addition).

The reference has no BERT (its encoder is the BiLSTM of model/graph.py:30-53); this module adds the
"FewRel 10-way 5-shot with BERT-base encoder" configuration of BASELINE.json.  Architecture =
BERT (post-LN transformer, GELU FFN) with HuggingFace parameter names and layouts (Linear weights
``[out, in]``), so a local HF checkpoint directory (``Config.bert_checkpoint``) is loaded by name
(``load_hf_state``; pinned to ``transformers.BertModel`` by tests/test_bert.py).
The sentence vector is pooled at the entity-start markers (concat of the [E1] and [E2] states) or
at [CLS], then projected to ``bert_out_dim`` -- the width the induction (routing) and relation
(NTN) heads run at (their fused kernels are instantiated for H in {16, 40, 64}).

This file holds the parameter table and the pure-PyTorch oracle (CPU path + kernel tests).  The
GPU path (ops/bert.py) runs the same math on hand-written gfx950 kernels (fused attention,
residual+dropout+LayerNorm, bias+GELU, embedding+LayerNorm) and hipBLASLt GEMMs.

Dropout uses the counter hash of models/reference.py (bit-identical to the kernels):
stream 16 = embedding output, 17 + 3*layer + {0: attention probs, 1: attention output,
2: FFN output}.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

from .reference import _M32

LN_EPS = 1e-12


def param_specs(cfg) -> "OrderedDict[str, Tuple[tuple, str]]":
    """HF name -> (shape, init) in flat-buffer order.  q/k/v weights (and biases) are adjacent so the
    flat bf16 copy exposes them as one [3*Hd, Hd] QKV matrix without a concat."""
    Hd, I, P = cfg.bert_hidden, cfg.bert_intermediate, cfg.bert_max_position
    V = cfg.bert_vocab
    sp = OrderedDict()
    e = "bert.embeddings."
    sp[e + "word_embeddings.weight"] = ((V, Hd), "normal")
    sp[e + "position_embeddings.weight"] = ((P, Hd), "normal")
    sp[e + "token_type_embeddings.weight"] = ((2, Hd), "normal")
    sp[e + "LayerNorm.weight"] = ((Hd,), "ones")
    sp[e + "LayerNorm.bias"] = ((Hd,), "zeros")
    for i in range(cfg.bert_layers):
        p = f"bert.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            sp[p + f"attention.self.{n}.weight"] = ((Hd, Hd), "normal")
        for n in ("query", "key", "value"):
            sp[p + f"attention.self.{n}.bias"] = ((Hd,), "zeros")
        sp[p + "attention.output.dense.weight"] = ((Hd, Hd), "normal")
        sp[p + "attention.output.dense.bias"] = ((Hd,), "zeros")
        sp[p + "attention.output.LayerNorm.weight"] = ((Hd,), "ones")
        sp[p + "attention.output.LayerNorm.bias"] = ((Hd,), "zeros")
        sp[p + "intermediate.dense.weight"] = ((I, Hd), "normal")
        sp[p + "intermediate.dense.bias"] = ((I,), "zeros")
        sp[p + "output.dense.weight"] = ((Hd, I), "normal")
        sp[p + "output.dense.bias"] = ((Hd,), "zeros")
        sp[p + "output.LayerNorm.weight"] = ((Hd,), "ones")
        sp[p + "output.LayerNorm.bias"] = ((Hd,), "zeros")
    pool = 2 * Hd if cfg.bert_pool == "entity" else Hd
    sp["bert_proj/kernel"] = ((pool, cfg.bert_out_dim), "glorot")
    sp["bert_proj/bias"] = ((cfg.bert_out_dim,), "zeros")
    return sp


def attr_of(name: str) -> str:
    return "bert__" + name.replace(".", "__").replace("/", "__")


def init_tensor(shape, kind: str, gen: torch.Generator) -> torch.Tensor:
    if kind == "normal":
        return torch.randn(shape, generator=gen) * 0.02
    if kind == "ones":
        return torch.ones(shape)
    if kind == "zeros":
        return torch.zeros(shape)
    if kind == "glorot":
        lim = math.sqrt(6.0 / (shape[0] + shape[1]))
        return (torch.rand(shape, generator=gen) * 2 - 1) * lim
    raise ValueError(kind)


# ------------------------------------------------------------------ dropout (hash shared with HIP)
def keep_mask(seed: int, stream: int, numel: int, keep_prob: float, device=None) -> torch.Tensor:
    """Bernoulli(keep_prob) float mask over flat indices 0..numel-1 (idx taken mod 2^32)."""
    idx = torch.arange(numel, dtype=torch.int64, device=device) & _M32
    salt = ((seed & 0x7FFFFFFF) * 0x2545F491 + stream * 0x3C6EF372 + 0x1234567) & _M32
    x = ((idx * 0x6C8E9CF5) & _M32) + salt
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    thr = min(int(keep_prob * 4294967296.0), 0xFFFFFFFF)
    return (x < thr).to(torch.float32)


def attn_keep_mask(seed: int, stream: int, S: int, nh: int, L: int, keep_prob: float, device=None) -> torch.Tensor:
    """Attention-probability keep mask [S, nh, L, L] (float 0/1): ONE hash per pair of adjacent keys.  Element
    (row, j), row = (s nh + h) L + i, keeps iff 16-bit half (j & 1) of mix(((row << 6) | (j >> 1)) * C + salt) is
    below floor(kp 2^32) >> 16 (csrc/kernels/bert.hip attn_mix; L <= 128)."""
    salt = ((seed & 0x7FFFFFFF) * 0x2545F491 + stream * 0x3C6EF372 + 0x1234567) & _M32
    row = torch.arange(S * nh * L, dtype=torch.int64, device=device)[:, None]
    j = torch.arange(L, dtype=torch.int64, device=device)[None, :]
    x = ((((row << 6) | (j >> 1)) * 0x6C8E9CF5) & _M32) + salt
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    v = torch.where((j & 1) == 1, x >> 16, x & 0xFFFF)
    thr16 = min(int(keep_prob * 4294967296.0), 0xFFFFFFFF) >> 16
    return (v < thr16).to(torch.float32).view(S, nh, L, L)


def _dropout(x: torch.Tensor, seed: int, stream: int, p: float, training: bool) -> torch.Tensor:
    if not training or p <= 0.0:
        return x
    kp = 1.0 - p
    m = keep_mask(seed, stream, x.numel(), kp, x.device).view_as(x)
    return x * m / kp


# ------------------------------------------------------------------ oracle layers
def gelu(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def layer_norm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + LN_EPS) * g + b


def attention(q, k, v, mask, nh: int, seed: int, stream: int, p: float, training: bool):
    """q/k/v [S, L, Hd]; mask [S, L] (1 = real key).  Dropout: attn_keep_mask (one hash per key pair)."""
    S, L, Hd = q.shape
    d = Hd // nh
    qh = q.view(S, L, nh, d).transpose(1, 2)
    kh = k.view(S, L, nh, d).transpose(1, 2)
    vh = v.view(S, L, nh, d).transpose(1, 2)
    sc = qh @ kh.transpose(-1, -2) / math.sqrt(d)
    sc = sc.masked_fill(mask[:, None, None, :] == 0, float("-inf"))
    pr = torch.softmax(sc, -1)
    if training and p > 0.0:
        pr = pr * attn_keep_mask(seed, stream, S, nh, L, 1.0 - p, pr.device) / (1.0 - p)
    return (pr @ vh).transpose(1, 2).reshape(S, L, Hd)


def encode_ref(p: Dict[str, torch.Tensor], ids, mask, e1, e2, cfg, training: bool = False,
               seed: int = 0) -> torch.Tensor:
    """Pure-PyTorch BERT encoder + pooling + projection -> [S, bert_out_dim] (fp32)."""
    x = hidden_states_ref(p, ids, mask, cfg, training, seed)
    return pool_project(p, x, e1, e2, cfg.bert_pool)


def hidden_states_ref(p: Dict[str, torch.Tensor], ids, mask, cfg, training: bool = False,
                      seed: int = 0) -> torch.Tensor:
    """The encoder's last hidden states [S, L, Hd] (HF ``BertModel(...).last_hidden_state``)."""
    S, L = ids.shape
    pd, ad = cfg.bert_dropout, cfg.bert_attn_dropout
    e = "bert.embeddings."
    x = (p[e + "word_embeddings.weight"][ids.long()] + p[e + "position_embeddings.weight"][:L][None]
         + p[e + "token_type_embeddings.weight"][0][None, None])
    x = layer_norm(x, p[e + "LayerNorm.weight"], p[e + "LayerNorm.bias"])
    x = _dropout(x, seed, 16, pd, training)
    for i in range(cfg.bert_layers):
        pre = f"bert.encoder.layer.{i}."
        a = pre + "attention."
        q = x @ p[a + "self.query.weight"].t() + p[a + "self.query.bias"]
        k = x @ p[a + "self.key.weight"].t() + p[a + "self.key.bias"]
        v = x @ p[a + "self.value.weight"].t() + p[a + "self.value.bias"]
        c = attention(q, k, v, mask, cfg.bert_heads, seed, 17 + 3 * i, ad, training)
        o = c @ p[a + "output.dense.weight"].t() + p[a + "output.dense.bias"]
        o = _dropout(o, seed, 18 + 3 * i, pd, training)
        x = layer_norm(x + o, p[a + "output.LayerNorm.weight"], p[a + "output.LayerNorm.bias"])
        h = gelu(x @ p[pre + "intermediate.dense.weight"].t() + p[pre + "intermediate.dense.bias"])
        o = h @ p[pre + "output.dense.weight"].t() + p[pre + "output.dense.bias"]
        o = _dropout(o, seed, 19 + 3 * i, pd, training)
        x = layer_norm(x + o, p[pre + "output.LayerNorm.weight"], p[pre + "output.LayerNorm.bias"])
    return x


def pool_project(p, x, e1, e2, pool: str) -> torch.Tensor:
    S = x.shape[0]
    ar = torch.arange(S, device=x.device)
    if pool == "entity":
        v = torch.cat([x[ar, e1.long()], x[ar, e2.long()]], -1)
    else:
        v = x[:, 0]
    return v.float() @ p["bert_proj/kernel"].float() + p["bert_proj/bias"].float()


def hf_names(cfg) -> List[str]:
    return [n for n in param_specs(cfg) if n.startswith("bert.")]


# ------------------------------------------------------------------ HF checkpoint import
def read_hf_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    """Tensors of a LOCAL HuggingFace checkpoint: a directory holding ``model.safetensors`` (or sharded
    ``model-*.safetensors``) or ``pytorch_model.bin``, or one such file.  Nothing that executes code
    is used: safetensors, or ``torch.load(weights_only=True)``."""
    import glob
    import os
    from safetensors.torch import load_file
    if os.path.isdir(path):
        st = sorted(glob.glob(os.path.join(path, "model*.safetensors")))
        if st:
            out: Dict[str, torch.Tensor] = {}
            for f in st:
                out.update(load_file(f))
            return out
        binf = os.path.join(path, "pytorch_model.bin")
        if not os.path.exists(binf):
            raise FileNotFoundError(f"no model*.safetensors or pytorch_model.bin in {path}")
        path = binf
    if path.endswith(".safetensors"):
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def hf_key_map(keys) -> Dict[str, str]:
    """checkpoint key -> our parameter name (``bert.`` prefixed HF names).  Accepts BertModel keys
    (``embeddings.*``, ``encoder.*``), task-model keys (``bert.*``) and the TF-converted LayerNorm
    names (``gamma`` / ``beta``); pooler / task-head keys are ignored."""
    out = {}
    for k in keys:
        n = k if k.startswith("bert.") else "bert." + k
        n = n.replace("LayerNorm.gamma", "LayerNorm.weight").replace("LayerNorm.beta", "LayerNorm.bias")
        if n.startswith(("bert.embeddings.", "bert.encoder.")):
            out[k] = n
    return out


def load_hf_state(params, path: str, cfg, strict: bool = True) -> List[str]:
    """Copy a local HF BERT checkpoint into ``params`` (models/params.py InductionParams, BERT mode).
    Every encoder tensor of our parameter table must be present with the same shape (``strict``), except
    that a checkpoint with more position embeddings than ``bert_max_position`` is cut to that length.
    The projection to ``bert_out_dim`` (``bert_proj/*``) is not part of BERT and keeps its init.
    Returns the loaded parameter names."""
    src = read_hf_checkpoint(path)
    km = hf_key_map(src.keys())
    by_name = {v: k for k, v in km.items()}
    loaded = []
    with torch.no_grad():
        for name in hf_names(cfg):
            dst = getattr(params, attr_of(name))
            if name not in by_name:
                if strict:
                    raise KeyError(f"BERT checkpoint {path} has no tensor for {name}")
                continue
            t = src[by_name[name]]
            if name.endswith("position_embeddings.weight") and t.shape[0] > dst.shape[0]:
                t = t[: dst.shape[0]]
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"BERT checkpoint {name}: shape {tuple(t.shape)} vs model {tuple(dst.shape)} "
                                 "(set bert_hidden / bert_layers / bert_heads / bert_intermediate / bert_vocab "
                                 "to the checkpoint's config)")
            dst.copy_(t.to(dst.device, dst.dtype))
            loaded.append(name)
    return loaded
