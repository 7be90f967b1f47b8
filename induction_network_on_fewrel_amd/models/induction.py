"""The Induction Network model (reference ``model/graph.py:15-109`` + ``model/base.py``).

GPU path (``device.type == 'cuda'``): two fused autograd functions over hand-written gfx950 kernels
  EncoderFn  -- embedding gather + BiLSTM + word-level self-attention  (ops/encoder.py)
  HeadFn     -- dynamic routing + neural tensor layer + sigmoid         (ops/head.py)
and no fallback: a missing kernel library raises.
CPU path: the pure-PyTorch oracle (models/reference.py), used for plumbing runs and tests.

N/K/Q are runtime arguments: only the reference head's ``w`` is N-dependent.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch
from torch import nn

from ..config import Config
from . import reference as ref
from .padding import SMALL_U, WIDE_U, next_width, padded_params, padding_enabled
from .params import InductionParams

GPU_SUPPORTED_U = (8, 20, 32)   # fused BiLSTM kernel instantiations; other widths use ops/wide.py


class InductionNetwork(nn.Module):
    def __init__(self, cfg: Config, word_vec_mat: Optional[np.ndarray] = None, vocab_size: Optional[int] = None,
                 seed: int = 0):
        super().__init__()
        cfg.validate()
        self.cfg = cfg
        self.params = InductionParams(cfg, word_vec_mat, vocab_size, seed)

    # ------------------------------------------------------------------
    def pdict(self) -> Dict[str, torch.Tensor]:
        return {a: getattr(self.params, a) for a in self.params.names()}

    def bert_pdict(self) -> Dict[str, torch.Tensor]:
        """HF name -> tensor view of the BERT encoder + projection parameters."""
        return {n: getattr(self.params, a) for a, n in self.params.names().items() if a.startswith("bert__")}

    def lstm_plan(self, L: int) -> Tuple[str, int]:
        """(path, width) of the GPU encoder: "small" = the fused lane-ownership BiLSTM+attention kernels
        (lstm.hip, u in {8, 20, 32}, input <= 64, L <= 64, pos dim <= 8), "wide" = ops/wide.py (persistent
        lstm_wide.hip kernels at u in {64, 100, 128}, the per-step GEMM loop otherwise).  A width between the
        instantiations runs exactly on the next one up with zero-padded parameters (models/padding.py;
        INA_LSTM_PAD=0 disables).  ``lstm_impl`` "fused" / "wide" forces the path."""
        cfg = self.cfg
        u, impl = cfg.hidden_size, cfg.lstm_impl
        small_ok = self.params.input_dim <= 64 and L <= 64 and cfg.pos_embedding_dim <= 8
        pad = padding_enabled()
        if impl != "wide":
            if small_ok and u in SMALL_U:
                return "small", u
            if small_ok and pad and u < SMALL_U[-1]:
                return "small", next_width(u, SMALL_U)
            if impl == "fused":
                raise NotImplementedError(f"fused BiLSTM kernels need u <= {SMALL_U[-1]} (instantiated for "
                                          f"{SMALL_U}), input dim <= 64, L <= 64, pos dim <= 8")
        if pad and u <= WIDE_U[-1] and u not in WIDE_U:
            return "wide", next_width(u, WIDE_U)
        return "wide", u

    def use_fused_lstm(self, L: int) -> bool:
        """The fused small-width kernels at the model's own width (the fused training step, graph capture)."""
        return self.lstm_plan(L) == ("small", self.cfg.hidden_size)

    def _head(self, e, p, B, N, K, Q, grad_views):
        """Fused routing + NTN kernels when instantiated for (H, N, Q), else the GEMM formulation."""
        cfg = self.cfg
        H = e.shape[1]
        if H in (16, 40, 64) and N <= 16 and N * Q <= 64:
            from ..ops.head import head
            return head(e, p, dict(E=B, N=N, K=K, Q=Q, iters=cfg.routing_iters,
                                   paper=(cfg.relation_head == "paper"), grad_views=grad_views))
        if e.is_cuda and cfg.dtype == "bf16":
            from ..ops.wide import head_wide
            return head_wide(e, p, B, N, K, Q, cfg.routing_iters, cfg.relation_head)
        return ref.head_forward(p, e.float(), B, N, K, Q, cfg.routing_iters, cfg.relation_head)

    def use_wide_head_loss(self, inst, data, N: int, K: int, Q: int) -> bool:
        """Training step through the wide head's fused loss node (head_wide.hip + ina.head_loss): GPU, bf16,
        a head shape outside the fused head kernels, and one the wide head kernels cover."""
        cfg = self.cfg
        if not (inst.is_cuda and cfg.dtype == "bf16"):
            return False
        H = int(self.params.head_dim)
        if H in (16, 40, 64) and N <= 16 and N * Q <= 64:
            return False
        from ..ops.wide import head_wide_ok
        return head_wide_ok(H, N, K, cfg.routing_iters, cfg.relation_head)

    def check_gpu_config(self, N: int, Q: int, L: int) -> None:
        u = self.cfg.hidden_size
        din = self.params.input_dim
        if u not in GPU_SUPPORTED_U:
            raise NotImplementedError(f"GPU kernels are instantiated for hidden_size in {GPU_SUPPORTED_U}, got {u}")
        if din > 64:
            raise NotImplementedError(f"GPU LSTM kernel supports input dim <= 64, got {din}")
        if L > 64:
            raise NotImplementedError(f"GPU attention kernel supports max_length <= 64, got {L}")
        if N > 16 or N * Q > 64:
            raise NotImplementedError("GPU NTN kernel supports N <= 16 and N*Q <= 64")

    def forward(self, inst: torch.Tensor, data: Tuple[torch.Tensor, ...], B: int, N: int, K: int, Q: int,
                training: bool = True, dropout_seed: int = 0,
                grad_views: Optional[Dict[str, torch.Tensor]] = None, overlap=None,
                seed_dev: Optional[torch.Tensor] = None, embeddings_only: bool = False, glue=None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """inst: int32 [B*(N*K+N*Q)] instance rows (episode layout, support first).
        data: (word, pos1, pos2, mask) [NI, L] int32 on the same device.
        Returns probs [B, N*Q, N] and alphas [B*(N*K+N*Q), L] (``embeddings_only``: the sentence
        vectors e [B*(N*K+N*Q), H] instead of probs; GPU path only)."""
        cfg = self.cfg
        kp = cfg.keep_prob if training else 1.0
        p = self.pdict()
        if self.cfg.relation_head == "reference" and p["ntn_w"].shape[1] != N:
            raise ValueError(f"reference relation head was built for N={p['ntn_w'].shape[1]}, got N={N} "
                             "(use relation_head='paper' for N-independent scoring)")
        if cfg.encoder == "bert":
            return self._forward_bert(inst, data, B, N, K, Q, training, dropout_seed, grad_views, p, overlap,
                                      embeddings_only, glue)
        if inst.is_cuda:
            word, pos1, pos2, mask = data
            path, up = self.lstm_plan(word.shape[1])
            u = cfg.hidden_size
            pe, real = (p, None) if up == u else padded_params(p, u, up, self.params.input_dim)
            if path == "small":
                from ..ops.encoder import encode
                meta = dict(U=up, bf16=(cfg.dtype == "bf16"), keep_prob=kp, seed=int(dropout_seed),
                            ragged=cfg.ragged_tiles, skip_padding=cfg.lstm_skip_padding,
                            word_grad=bool(isinstance(p["word_embedding"], nn.Parameter)
                                           and p["word_embedding"].requires_grad),
                            grad_views=grad_views if real is None else None, seed_dev=seed_dev)
                e, alphas = encode(inst, data, pe, meta)
            else:   # wide layers (e.g. the paper's u=128, E=300): persistent kernels or the GEMM loop
                from ..ops.wide import encode_wide
                if cfg.lstm_skip_padding:
                    raise NotImplementedError("lstm_skip_padding: the wide GPU path runs the reference's full L")
                # training with the step glue: the kernel path's gradients go to its scatter-add (flat parameters only)
                gl = glue if (training and glue is not None and grad_views is not None and real is None) else None
                e, alphas = encode_wide(inst, data, pe, up, kp, int(dropout_seed), glue=gl)
            if real is not None:   # the real units of the zero-padded encoder
                e = e[:, real]
            if embeddings_only:
                return e, alphas
            return self._head(e, p, B, N, K, Q, grad_views), alphas
        word, pos1, pos2, mask = (t[inst.long()] for t in data)
        probs, alphas = ref.forward(p, word, pos1, pos2, mask, B, N, K, Q, cfg.routing_iters, cfg.relation_head,
                                    kp, int(dropout_seed), bf16=False, skip_padding=cfg.lstm_skip_padding)
        return probs, alphas.squeeze(-1)

    def _forward_bert(self, inst, data, B, N, K, Q, training, dropout_seed, grad_views, p, overlap=None,
                      embeddings_only=False, glue=None):
        """BERT encoder (data = (ids, mask, e1, e2) [NI, Lb] int32) + the same induction/relation head.
        Returns probs and the [CLS]-row attention-free placeholder alphas (None)."""
        cfg = self.cfg
        if inst.is_cuda:
            from ..ops.bert import bert_encode
            e = bert_encode(self, inst, data, training, int(dropout_seed), grad_views, overlap,
                            glue if training else None)
            if embeddings_only:
                return e, None
            return self._head(e, p, B, N, K, Q, grad_views), None
        from . import bert as Bm
        ids, mask, e1, e2 = (t[inst.long()] for t in data)
        e = Bm.encode_ref(self.bert_pdict(), ids, mask, e1, e2, cfg, training, int(dropout_seed))
        probs = ref.head_forward(p, e, B, N, K, Q, cfg.routing_iters, cfg.relation_head)
        return probs, None

    def forward_train(self, inst: torch.Tensor, data: Tuple[torch.Tensor, ...], B: int, N: int, K: int, Q: int,
                      labels: torch.Tensor, dropout_seed: int = 0,
                      grad_views: Optional[Dict[str, torch.Tensor]] = None, overlap=None,
                      seed_dev: Optional[torch.Tensor] = None, glue=None):
        """Training forward with the loss: -> (loss, accuracy, probs).

        With a ``StepGlue`` on the fused GPU BiLSTM path this is the low-launch step (one pack
        gather, encoder, routing/NTN/loss in one node; gradients queued for the glue's single
        scatter-add -- the caller runs ``glue.flush()`` after backward).  Otherwise it is
        forward + ``loss`` + ``accuracy`` (CPU, BERT, wide layers, GEMM-formulated head)."""
        cfg = self.cfg
        p = self.pdict()
        H = 2 * cfg.hidden_size
        fused = (glue is not None and inst.is_cuda and cfg.encoder == "bilstm" and grad_views is not None
                 and self.use_fused_lstm(data[0].shape[1]) and H in (16, 40, 64) and N <= 16 and N * Q <= 64
                 and not (cfg.relation_head == "reference" and p["ntn_w"].shape[1] != N))
        if not fused and self.use_wide_head_loss(inst, data, N, K, Q):
            from ..ops.wide import head_wide_loss
            e, _ = self.forward(inst, data, B, N, K, Q, training=True, dropout_seed=dropout_seed,
                                grad_views=grad_views, overlap=overlap, seed_dev=seed_dev, embeddings_only=True,
                                glue=glue)
            return head_wide_loss(e, p, labels, B, N, K, Q, cfg.routing_iters, cfg.relation_head, cfg.loss_type,
                                  cfg.loss_reduction, glue=glue if grad_views is not None else None)
        if not fused:
            probs, _ = self.forward(inst, data, B, N, K, Q, training=True, dropout_seed=dropout_seed,
                                    grad_views=grad_views, overlap=overlap, seed_dev=seed_dev, glue=glue)
            loss = self.loss(probs, labels)
            with torch.no_grad():   # ce_nota: a query is predicted NOTA below the score 0.5 (its loss's NOTA class)
                acc = ref.accuracy(probs.detach(), labels.long(), 0.5 if cfg.loss_type == "ce_nota" else None)
            return loss, acc, probs
        from ..ops.encoder import encode
        from ..ops.glue import lstm_din
        from ..ops.head import head_loss
        U, bf16 = cfg.hidden_size, cfg.dtype == "bf16"
        paper = cfg.relation_head == "paper"
        packs = glue.packs(p, U, lstm_din(p), bf16, (H, p["M"].shape[2], N, paper))
        meta = dict(U=U, bf16=bf16, keep_prob=cfg.keep_prob, seed=int(dropout_seed), ragged=cfg.ragged_tiles,
                    skip_padding=cfg.lstm_skip_padding, word_grad=bool(isinstance(p["word_embedding"], nn.Parameter) and p["word_embedding"].requires_grad),
                    grad_views=grad_views, seed_dev=seed_dev, packs=packs, glue=glue, pdict=p)
        e, _ = encode(inst, data, p, meta)
        return head_loss(e, p, labels, dict(E=B, N=N, K=K, Q=Q, iters=cfg.routing_iters, paper=paper, glue=glue,
                                            packs=packs, pdict=p, reduction=cfg.loss_reduction,
                                            loss_type=cfg.loss_type, overlap=overlap))

    # ------------------------------------------------------------------
    def loss(self, probs: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        return ref.loss_fn(self.cfg.loss_type)(probs, labels.long(), self.cfg.loss_reduction)

    def l2_value(self) -> torch.Tensor:
        return sum((v.detach() ** 2).sum() / 2 for v in self.params.l2_vars()) * self.cfg.l2_lambda
