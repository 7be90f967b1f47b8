"""Trainable state of the Induction Network, keyed by the reference's TF1 variable names.

Name/shape/init table = SURVEY 2.4 (derived from ``model/base.py:38-74``,
``model/graph.py:34-44``, ``model/layer_module.py:16-17,39-42,61-72,116-119``):

=============================================  ==================  =====================
TF name                                        shape               init
=============================================  ==================  =====================
embedding/Variable  (pretrained, frozen)       [V+2, E]            GloVe, L2-normed
word_embedding      (no pretrained table)      [vocab, E]          N(0, 0.1)
pos1_embedding, pos2_embedding                 [2L, 5]             N(0, 0.1)
bidirectional_rnn/{fw,bw}/basic_lstm_cell/kernel [E+10+u, 4u]      glorot-uniform
bidirectional_rnn/{fw,bw}/basic_lstm_cell/bias   [4u]              zeros
self_attn/dense/kernel, self_attn/dense/bias   [2u,2u], [2u]       glorot-uniform, zeros
self_attn/W_a2                                 [2u, 1]             glorot-normal
W_s                                            [2u, 2u]            glorot-normal
M                                              [2u, 2u, h]         glorot-normal
w                                              [h*N, N]            glorot-normal
b                                              [N]                 glorot-normal
=============================================  ==================  =====================

LSTM kernel gate column order is TF ``BasicLSTMCell``: i, j, f, o; input rows [x_t ; h_{t-1}].
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch
from torch import nn

from ..config import Config


def _fans(shape):
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = 1
    for d in shape[:-2]:
        rf *= d
    return shape[-2] * rf, shape[-1] * rf


def glorot_uniform_(t: torch.Tensor, gen: torch.Generator) -> torch.Tensor:
    fi, fo = _fans(tuple(t.shape))
    lim = math.sqrt(6.0 / (fi + fo))
    with torch.no_grad():
        t.copy_((torch.rand(t.shape, generator=gen) * 2 - 1) * lim)
    return t


def glorot_normal_(t: torch.Tensor, gen: torch.Generator) -> torch.Tensor:
    """TF1 ``glorot_normal``: truncated normal (|z|<2), std = sqrt(2/(fi+fo))/0.87962566."""
    fi, fo = _fans(tuple(t.shape))
    std = math.sqrt(2.0 / (fi + fo)) / 0.87962566103423978
    with torch.no_grad():
        z = torch.randn(t.shape, generator=gen)
        bad = z.abs() >= 2
        while bool(bad.any()):
            z[bad] = torch.randn(int(bad.sum()), generator=gen)
            bad = z.abs() >= 2
        t.copy_(z * std)
    return t


def normal_(t: torch.Tensor, gen: torch.Generator, std: float) -> torch.Tensor:
    with torch.no_grad():
        t.copy_(torch.randn(t.shape, generator=gen) * std)
    return t


# attribute name -> TF variable name
TF_NAMES = OrderedDict([
    ("word_embedding", None),  # resolved per instance (pretrained vs trainable)
    ("pos1_embedding", "pos1_embedding"),
    ("pos2_embedding", "pos2_embedding"),
    ("lstm_fw_kernel", "bidirectional_rnn/fw/basic_lstm_cell/kernel"),
    ("lstm_fw_bias", "bidirectional_rnn/fw/basic_lstm_cell/bias"),
    ("lstm_bw_kernel", "bidirectional_rnn/bw/basic_lstm_cell/kernel"),
    ("lstm_bw_bias", "bidirectional_rnn/bw/basic_lstm_cell/bias"),
    ("attn_kernel", "self_attn/dense/kernel"),
    ("attn_bias", "self_attn/dense/bias"),
    ("attn_w2", "self_attn/W_a2"),
    ("W_s", "W_s"),
    ("M", "M"),
    ("ntn_w", "w"),
    ("ntn_b", "b"),
])


class InductionParams(nn.Module):
    """All trainable + frozen tensors. Parameters are fp32 masters."""

    def __init__(self, cfg: Config, word_vec_mat: Optional[np.ndarray] = None, vocab_size: Optional[int] = None,
                 seed: int = 0):
        super().__init__()
        self.cfg = cfg
        gen = torch.Generator().manual_seed(seed)
        h = cfg.ntn_slices
        N = cfg.N
        # attr -> checkpoint name, in flat-buffer order
        self._names: "OrderedDict[str, str]" = OrderedDict()
        self.pretrained = False
        if cfg.encoder == "bert":
            from . import bert as B
            for name, (shape, kind) in B.param_specs(cfg).items():
                a = B.attr_of(name)
                setattr(self, a, nn.Parameter(B.init_tensor(shape, kind, gen)))
                self._names[a] = name
            if cfg.bert_checkpoint:   # a local HF checkpoint (safetensors / weights-only torch file)
                B.load_hf_state(self, cfg.bert_checkpoint, cfg)
            H = cfg.bert_out_dim
            self.word_dim = cfg.bert_hidden
            self.input_dim = cfg.bert_hidden
        else:
            L, u, pd = cfg.max_length, cfg.hidden_size, cfg.pos_embedding_dim
            H = 2 * u
            if word_vec_mat is not None:
                wv = torch.as_tensor(np.asarray(word_vec_mat, dtype=np.float32))
                self.pretrained = True
                if cfg.train_word_embedding:
                    self.word_embedding = nn.Parameter(wv.clone())
                else:
                    self.register_buffer("word_embedding", wv.clone())
            else:
                if vocab_size is None:
                    raise ValueError("need word_vec_mat or vocab_size")
                self.word_embedding = nn.Parameter(normal_(torch.empty(vocab_size, cfg.synthetic_word_dim), gen,
                                                           cfg.init_std))
            E = self.word_embedding.shape[1]
            self.word_dim = E
            D = E + 2 * pd
            self.input_dim = D
            self.pos1_embedding = nn.Parameter(normal_(torch.empty(2 * L, pd), gen, cfg.init_std))
            self.pos2_embedding = nn.Parameter(normal_(torch.empty(2 * L, pd), gen, cfg.init_std))
            self.lstm_fw_kernel = nn.Parameter(glorot_uniform_(torch.empty(D + u, 4 * u), gen))
            self.lstm_fw_bias = nn.Parameter(torch.zeros(4 * u))
            self.lstm_bw_kernel = nn.Parameter(glorot_uniform_(torch.empty(D + u, 4 * u), gen))
            self.lstm_bw_bias = nn.Parameter(torch.zeros(4 * u))
            self.attn_kernel = nn.Parameter(glorot_uniform_(torch.empty(H, H), gen))
            self.attn_bias = nn.Parameter(torch.zeros(H))
            self.attn_w2 = nn.Parameter(glorot_normal_(torch.empty(H, 1), gen))
            for a in list(TF_NAMES)[:10]:
                self._names[a] = ("embedding/Variable" if self.pretrained else "word_embedding") \
                    if a == "word_embedding" else TF_NAMES[a]
        self.head_dim = H
        self.W_s = nn.Parameter(glorot_normal_(torch.empty(H, H), gen))
        self.M = nn.Parameter(glorot_normal_(torch.empty(H, H, h), gen))
        if cfg.relation_head == "reference":
            self.ntn_w = nn.Parameter(glorot_normal_(torch.empty(h * N, N), gen))
            self.ntn_b = nn.Parameter(glorot_normal_(torch.empty(N), gen))
        else:
            self.ntn_w = nn.Parameter(glorot_normal_(torch.empty(h, 1), gen))
            self.ntn_b = nn.Parameter(glorot_normal_(torch.empty(1), gen))
        for a in ("W_s", "M", "ntn_w", "ntn_b"):
            self._names[a] = TF_NAMES[a]

    # ------------------------------------------------------------ naming
    def names(self) -> "OrderedDict[str, str]":
        """attr -> checkpoint name (TF1 names for the BiLSTM model, HF names for BERT)."""
        return self._names

    def tf_name(self, attr: str) -> str:
        return self._names[attr]

    def tf_state(self) -> "OrderedDict[str, torch.Tensor]":
        out = OrderedDict()
        for attr, name in self._names.items():
            out[name] = getattr(self, attr).detach()
        return out

    def load_tf_state(self, state: Dict[str, torch.Tensor], strict: bool = True) -> None:
        with torch.no_grad():
            for attr, name in self._names.items():
                if name not in state:
                    if strict:
                        raise KeyError(f"missing {name} in checkpoint")
                    continue
                dst = getattr(self, attr)
                src = state[name]
                if tuple(src.shape) != tuple(dst.shape):
                    raise ValueError(f"shape mismatch for {name}: {tuple(src.shape)} vs {tuple(dst.shape)}")
                dst.copy_(src.to(dst.device, dst.dtype))

    def trainable(self) -> "OrderedDict[str, nn.Parameter]":
        """Ordered (attr -> Parameter) of trainable tensors (the flat-buffer order)."""
        out = OrderedDict()
        for attr in self._names:
            t = getattr(self, attr)
            if isinstance(t, nn.Parameter) and t.requires_grad:
                out[attr] = t
        return out

    def l2_vars(self):
        """Vars the reference's (dead) L2 term covers (graph.py:98-106): names without 'bias',
        'word_embedding', 'pos1_embedding', 'pos2_embedding'. Note the NTN bias is named ``b``
        so the reference *does* regularise it."""
        out = []
        for a, p in self.trainable().items():
            n = self.tf_name(a)
            if ("bias" in n or "word_embedding" in n or "pos1_embedding" in n or "pos2_embedding" in n
                    or "embeddings" in n or "LayerNorm" in n):
                continue
            out.append(p)
        return out
