"""Exact zero-padding of the BiLSTM + self-attention encoder to a width the persistent kernels are built for.

The reference's ``hidden_size`` is a free knob (/root/reference/model/base.py:16, train.py:36), while the
persistent gfx950 BiLSTM kernels are instantiated for u in {8, 20, 32} (lstm.hip) and {64, 100, 128}
(lstm_wide.hip).  Any other u <= 128 runs on the next instantiated width Up > u with the parameters embedded
in zero-padded tensors (differentiable, so autograd returns the gradient of the real slice):

* LSTM kernel [D + u, 4u] -> [D + Up, 4Up]: every gate block (i, j, f, o) keeps its u columns first, the
  Up - u padded columns and the padded recurrent-input rows are zero; bias likewise.
* A padded unit has zero pre-activations, so c = f c_prev + i tanh(0) stays 0 from c_0 = 0 and h = o tanh(0)
  = 0 at every step (the forget bias only scales the zero cell); it feeds nothing back (zero rows of W_h).
* attention W1 [2u, 2u], b1, w2: the padded rows / columns are zero, so the projection, the scores and the
  pooled real columns are unchanged; the pooled vector is gathered back to [fw 0..u-1, bw 0..u-1].
* Backward: dh of a padded unit is 0 (zero W1 rows, its pooled column is dropped), so every gate gradient
  of a padded unit is 0 and the real units' gradients equal the unpadded network's.

The output dropout (DropoutWrapper) hashes (sequence, step, unit) over the PADDED width, so at keep_prob < 1
the real units' masks are a different (equally distributed) draw than an unpadded run: exact vs the oracle
at keep_prob = 1, and vs the oracle run on the padded parameters at any keep_prob (tests/test_wide_gpu.py).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

SMALL_U = (8, 20, 32)     # lstm.hip instantiations
WIDE_U = (64, 100, 128)   # lstm_wide.hip instantiations


def padding_enabled() -> bool:
    return os.environ.get("INA_LSTM_PAD", "1") != "0"


def next_width(u: int, widths) -> Optional[int]:
    for w in widths:
        if w >= u:
            return w
    return None


def _real_index(u: int, up: int, device) -> torch.Tensor:
    """Positions of the real units in a padded [fw | bw] vector of width 2 up."""
    r = torch.arange(u, device=device)
    return torch.cat([r, r + up])


def pad_lstm_kernel(k: torch.Tensor, u: int, up: int, d: int) -> torch.Tensor:
    """[d + u, 4u] -> [d + up, 4up] (gate blocks kept in order, zero padded columns / recurrent rows)."""
    g = k.view(d + u, 4, u)
    g = torch.nn.functional.pad(g, (0, up - u))                       # [d + u, 4, up]
    g = torch.cat([g, g.new_zeros(up - u, 4, up)], 0)                 # [d + up, 4, up]
    return g.reshape(d + up, 4 * up)


def pad_lstm_bias(b: torch.Tensor, u: int, up: int) -> torch.Tensor:
    return torch.nn.functional.pad(b.view(4, u), (0, up - u)).reshape(4 * up)


def pad_attention(w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, u: int, up: int):
    idx = _real_index(u, up, w1.device)
    h = 2 * up
    w1p = w1.new_zeros(h, h).index_put((idx.view(-1, 1), idx.view(1, -1)), w1)
    b1p = b1.new_zeros(h).index_put((idx,), b1)
    w2p = w2.new_zeros(h, w2.shape[1]).index_put((idx,), w2)
    return w1p, b1p, w2p


def padded_params(p: Dict[str, torch.Tensor], u: int, up: int, d: int) -> Tuple[Dict[str, torch.Tensor], torch.Tensor]:
    """A copy of the parameter dict with the encoder tensors padded to width up, and the index of the real
    columns of the padded sentence vector."""
    q = dict(p)
    for side in ("fw", "bw"):
        q[f"lstm_{side}_kernel"] = pad_lstm_kernel(p[f"lstm_{side}_kernel"], u, up, d)
        q[f"lstm_{side}_bias"] = pad_lstm_bias(p[f"lstm_{side}_bias"], u, up)
    q["attn_kernel"], q["attn_bias"], q["attn_w2"] = pad_attention(p["attn_kernel"], p["attn_bias"], p["attn_w2"],
                                                                  u, up)
    return q, _real_index(u, up, p["attn_kernel"].device)
