"""Pure-PyTorch oracle of the Induction Network with the reference's exact TF1 semantics.

This is the CPU execution path (BASELINE config 1, world_size=1 plumbing) and the
numerics oracle every HIP kernel is tested against. It is *not* used on the GPU path.

Semantics reproduced:
* embedding concat [word ; pos1 ; pos2]                           -- model/base.py:76-86
* BiLSTM, TF BasicLSTMCell gate order i,j,f,o, forget_bias 1.0, full L steps (no
  sequence_length), output-only dropout (DropoutWrapper)          -- model/graph.py:34-49
* self-attention pooling with the ``(1-mask)*(-2^31)`` adder on ``mask>0``
                                                                  -- layer_module.py:49-98, graph.py:52
* dynamic routing, shared W_s without bias, 3 iterations, squash  -- layer_module.py:101-162
* neural tensor layer with the ``s*N + c`` column order, ReLU, FC [h*N, N] + sigmoid
                                                                  -- layer_module.py:8-47
* MSE *mean* against one_hot(label, N)                            -- graph.py:92-94
* argmax accuracy                                                 -- base.py:101-107

``emulate_bf16`` rounds exactly the operands the HIP kernels feed to bf16 MFMAs, so the
oracle can check the bf16 kernels tightly.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

MASK_ADDER = -(2.0 ** 31)


def _r(x: torch.Tensor, on: bool) -> torch.Tensor:
    return x.to(torch.bfloat16).to(x.dtype) if on else x


# ------------------------------------------------------------------ dropout RNG
_M32 = 0xFFFFFFFF


def hash_u32(x: torch.Tensor) -> torch.Tensor:
    """Counter-based 32-bit hash; identical integer recipe to ``csrc/include/ina_common.h``.
    Constants < 2^31 so every product fits int64 exactly."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x68E31DA4) & _M32
    x = x ^ (x >> 16)
    return x


def dropout_keep_mask(seed: int, direction: int, S: int, L: int, u: int, keep_prob: float,
                      device=None) -> torch.Tensor:
    """Bernoulli(keep_prob) mask [S, L, u] for one LSTM direction's outputs (float 0/1).
    Same integer recipe as ``lstm_keep`` in csrc/include/ina_common.h: one 32-bit hash per pair of
    adjacent units (element e uses 16-bit half e & 1 of mix(e >> 1)), kept iff the half is below
    thr >> 16 (products are reduced mod 2^32 after every multiply; int64 never overflows)."""
    e = torch.arange(S * L * u, dtype=torch.int64, device=device)
    salt = ((seed & 0x7FFFFFFF) * 0x2545F491 + direction * 0x3C6EF372 + 0x1234567) & _M32
    x = ((e >> 1) * 0x6C8E9CF5 + salt) & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    thr16 = min(int(keep_prob * 4294967296.0), 0xFFFFFFFF) >> 16
    half = torch.where((e & 1) == 1, x >> 16, x & 0xFFFF)
    return (half < thr16).to(torch.float32).view(S, L, u)


# ------------------------------------------------------------------ encoder
def embed(word_emb, pos1_emb, pos2_emb, word, pos1, pos2) -> torch.Tensor:
    return torch.cat([word_emb[word], pos1_emb[pos1], pos2_emb[pos2]], dim=-1)


def lstm_direction(x: torch.Tensor, kernel: torch.Tensor, bias: torch.Tensor, reverse: bool,
                   bf16: bool = False, lengths: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (h_all, c_all) [S, L, u] in *time* order (bw outputs re-reversed).

    ``lengths`` (opt-in ``lstm_skip_padding``): TF ``dynamic_rnn(sequence_length=...)`` semantics -- at
    t >= length the output is zero and the state is carried unchanged, so the backward direction starts
    at length - 1 from the zero state.  None = the reference: every L step, padding included
    (model/graph.py:44-47)."""
    S, L, _ = x.shape
    u = kernel.shape[1] // 4
    h = x.new_zeros(S, u)
    c = x.new_zeros(S, u)
    W = _r(kernel, bf16)
    hs, cs = [None] * L, [None] * L
    steps = range(L - 1, -1, -1) if reverse else range(L)
    for t in steps:
        xh = torch.cat([_r(x[:, t], bf16), _r(h, bf16)], dim=-1)
        g = xh @ W + bias
        i, j, f, o = g.split(u, dim=-1)
        c_new = c * torch.sigmoid(f + 1.0) + torch.sigmoid(i) * torch.tanh(j)
        h_new = torch.tanh(c_new) * torch.sigmoid(o)
        if lengths is None:
            h, c = h_new, c_new
            hs[t], cs[t] = h, c
        else:
            m = (t < lengths).to(x.dtype).unsqueeze(-1)
            h = m * h_new + (1 - m) * h
            c = m * c_new + (1 - m) * c
            hs[t], cs[t] = m * h, m * c
    return torch.stack(hs, 1), torch.stack(cs, 1)


def valid_lengths(mask: torch.Tensor) -> torch.Tensor:
    """Per row: 1 + the last position with mask > 0 (0 for an all-padding row)."""
    L = mask.shape[-1]
    pos = torch.arange(1, L + 1, device=mask.device).expand_as(mask)
    return torch.where(mask > 0, pos, torch.zeros_like(pos)).amax(-1)


def self_attention(Hin: torch.Tensor, mask01: torch.Tensor, kernel, bias, w2, bf16: bool = False):
    """Hin [S, L, H], mask01 [S, L] (1 = attend). Returns (e [S, H], alphas [S, L, 1])."""
    proj = torch.tanh(_r(Hin, bf16) @ _r(kernel, bf16) + bias)
    score = proj @ w2                                  # [S, L, 1]
    adder = (1.0 - mask01.to(score.dtype)).unsqueeze(-1) * MASK_ADDER
    alphas = torch.softmax(score + adder, dim=1)
    e = torch.matmul(Hin.transpose(1, 2), alphas).squeeze(-1)
    return e, alphas


def encode(p: Dict[str, torch.Tensor], word, pos1, pos2, mask, keep_prob: float = 1.0,
           dropout_seed: int = 0, bf16: bool = False, return_all: bool = False, skip_padding: bool = False):
    """Sentence encoder: [S, L] id arrays -> e [S, 2u] (+ alphas).  ``skip_padding``: the BiLSTM gets
    sequence lengths (``lstm_skip_padding``; the reference runs through the padding)."""
    x = embed(p["word_embedding"], p["pos1_embedding"], p["pos2_embedding"], word, pos1, pos2)
    lens = valid_lengths(mask) if skip_padding else None
    hf, cf = lstm_direction(x, p["lstm_fw_kernel"], p["lstm_fw_bias"], False, bf16, lens)
    hb, cb = lstm_direction(x, p["lstm_bw_kernel"], p["lstm_bw_bias"], True, bf16, lens)
    if bf16:   # kernels store the LSTM outputs as bf16
        hf, hb = _r(hf, True), _r(hb, True)
    if keep_prob < 1.0:
        S, L, u = hf.shape
        mf = dropout_keep_mask(dropout_seed, 0, S, L, u, keep_prob, hf.device)
        mb = dropout_keep_mask(dropout_seed, 1, S, L, u, keep_prob, hf.device)
        hf = hf * mf / keep_prob
        hb = hb * mb / keep_prob
    Hin = torch.cat([hf, hb], dim=-1)
    e, alphas = self_attention(Hin, (mask > 0), p["attn_kernel"], p["attn_bias"], p["attn_w2"], bf16)
    if return_all:
        return e, alphas, {"x": x, "hf": hf, "hb": hb, "cf": cf, "cb": cb, "H": Hin}
    return e, alphas


# ------------------------------------------------------------------ induction
def squash(v: torch.Tensor) -> torch.Tensor:
    n = (v * v).sum(-1, keepdim=True)
    return v * (n / (1 + n) / torch.sqrt(n + 1e-9))


def dynamic_routing(sup: torch.Tensor, W_s: torch.Tensor, iters: int = 3) -> torch.Tensor:
    """sup [B, N, K, H] -> class vectors [B, N, H]."""
    e_hat = sup @ W_s
    b = sup.new_zeros(sup.shape[:-1])
    c = None
    for _ in range(iters):
        d = torch.softmax(b, dim=-1)
        c_hat = (d.unsqueeze(-1) * e_hat).sum(-2)
        c = squash(c_hat)
        b = b + (e_hat * c.unsqueeze(-2)).sum(-1)
    return c


# ------------------------------------------------------------------ relation
def ntn_features(cls: torch.Tensor, qry: torch.Tensor, M: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    """T[b, q, s, c] = sum_{a,b'} C[c,a] M[a,b',s] Q[q,b']  (pre-ReLU)."""
    P = torch.einsum("bna,ahs->bnhs", _r(cls, bf16), _r(M, bf16))           # [B, N, H, h]
    if bf16:
        P = _r(P, True)
    return torch.einsum("bqh,bnhs->bqsn", _r(qry, bf16), P)               # [B, NQ, h, N]


def relation_probs(cls, qry, M, w, b, head: str = "reference", bf16: bool = False) -> torch.Tensor:
    T = ntn_features(cls, qry, M, bf16)
    V = torch.relu(T)
    B, NQ, h, N = V.shape
    if head == "reference":
        logits = _r(V, bf16).reshape(B, NQ, h * N) @ _r(w, bf16) + b      # column index s*N + c
    else:
        logits = torch.einsum("bqsn,s->bqn", V, w[:, 0]) + b
    return torch.sigmoid(logits)


def one_hot_nota(labels: torch.Tensor, N: int) -> torch.Tensor:
    """tf.one_hot semantics: an out-of-range label (NOTA == N) gives an all-zero row."""
    return (labels.unsqueeze(-1) == torch.arange(N, device=labels.device)).to(torch.float32)


def mse_loss(probs: torch.Tensor, labels: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    y = one_hot_nota(labels, probs.shape[-1])
    d = (y - probs) ** 2
    return d.mean() if reduction == "mean" else d.sum() / max(1, probs.shape[0])


CE_ODDS_EPS = 1e-7   # 1 - p floor when recovering the logit from a saturated sigmoid (same in glue.hip)
CE_P_MIN = 1e-30     # p floor: z >= -69, never -inf (an underflowed sigmoid would give inf / NaN losses)


def relation_logits(probs: torch.Tensor) -> torch.Tensor:
    """Pre-sigmoid relation scores z = log p - log(1 - p), exact for z in [-69, 16.1]; outside it the
    clamps saturate z (and stop its gradient): a score already that confident is not pushed further."""
    return torch.log(torch.clamp(probs, min=CE_P_MIN)) - torch.log(torch.clamp(1.0 - probs, min=CE_ODDS_EPS))


def ce_loss(probs: torch.Tensor, labels: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """Softmax cross-entropy over the N relation scores of each query (``loss_type='ce'``, an
    opt-in alternative to the reference's MSE-on-sigmoid).  NOTA queries (label == N) carry no
    class to score and contribute zero loss.  ``mean``: over the labelled queries; ``sum``: summed
    and divided by the episode count (like ``mse_loss``)."""
    N = probs.shape[-1]
    z = relation_logits(probs).reshape(-1, N)
    lab = labels.reshape(-1).long()
    keep = lab < N
    nll = torch.nn.functional.cross_entropy(z, torch.where(keep, lab, torch.zeros_like(lab)), reduction="none")
    nll = nll * keep.to(nll.dtype)
    if reduction == "mean":
        return nll.sum() / max(1, int(lab.numel()))
    return nll.sum() / max(1, probs.shape[0])


def ce_nota_loss(probs: torch.Tensor, labels: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """NOTA-aware softmax cross-entropy (``loss_type='ce_nota'``, FewRel 2.0 training with none-of-the-above
    queries; no reference counterpart): the softmax runs over the N relation logits plus a NOTA class whose logit
    is fixed at 0 (relation score 0.5), and a NOTA query (label == N) targets that class.  ``mean`` over all
    queries; ``sum`` divided by the episode count."""
    N = probs.shape[-1]
    z = relation_logits(probs).reshape(-1, N)
    z = torch.cat([z, torch.zeros_like(z[:, :1])], 1)
    nll = torch.nn.functional.cross_entropy(z, labels.reshape(-1).long(), reduction="sum")
    return nll / max(1, int(labels.numel())) if reduction == "mean" else nll / max(1, probs.shape[0])


LOSS_MODES = {"mse": 0, "ce": 1, "ce_nota": 2}   # the fused loss kernel's mode (glue.hip head_loss)


def loss_fn(loss_type: str):
    return {"mse": mse_loss, "ce": ce_loss, "ce_nota": ce_nota_loss}[loss_type]


def predict(probs: torch.Tensor, nota_threshold: Optional[float] = None) -> torch.Tensor:
    pred = probs.argmax(-1)
    if nota_threshold is not None:
        N = probs.shape[-1]
        pred = torch.where(probs.max(-1).values < nota_threshold, torch.full_like(pred, N), pred)
    return pred


def accuracy(probs: torch.Tensor, labels: torch.Tensor, nota_threshold: Optional[float] = None) -> torch.Tensor:
    return (predict(probs, nota_threshold) == labels).to(torch.float32).mean()


# ------------------------------------------------------------------ full model
def forward(p: Dict[str, torch.Tensor], word, pos1, pos2, mask, B: int, N: int, K: int, Q: int,
            routing_iters: int = 3, head: str = "reference", keep_prob: float = 1.0, dropout_seed: int = 0,
            bf16: bool = False, skip_padding: bool = False):
    """Episode batch forward. Row layout per episode: [support N*K ; query N*Q]."""
    e, alphas = encode(p, word, pos1, pos2, mask, keep_prob, dropout_seed, bf16, skip_padding=skip_padding)
    return head_forward(p, e, B, N, K, Q, routing_iters, head, bf16), alphas


def head_forward(p: Dict[str, torch.Tensor], e, B: int, N: int, K: int, Q: int, routing_iters: int = 3,
                 head: str = "reference", bf16: bool = False):
    """Routing + relation head over sentence vectors e [B*(N*K+N*Q), H] -> probs [B, N*Q, N]."""
    H = e.shape[-1]
    e = e.view(B, N * K + N * Q, H)
    sup = e[:, : N * K].reshape(B, N, K, H)
    qry = e[:, N * K:]
    cls = dynamic_routing(sup, p["W_s"], routing_iters)
    return relation_probs(cls, qry, p["M"], p["ntn_w"], p["ntn_b"], head, bf16)
