"""Episodic trainer / evaluator (reference ``Base.train`` / ``Base.eval``, model/base.py:115-208).

Cadence kept from the reference: ``train_iter`` steps, running loss/acc printed every ``log_every``
(100) steps and reset at ``it % val_step == 0``; validation every ``val_step`` (2000) steps over
``val_iter`` (1000) episodes; checkpoint on best val accuracy; final "test" over ``test_iter`` (3000)
episodes of the val loader (the reference has no test split).

Fixes / additions (flagged in SURVEY 2.7): eval feeds the mask (#1) and is forward-only; resume from
the latest checkpoint (5.4); B episodes per step; rank-folded samplers + flat-buffer all-reduce (DP);
NaN/Inf loss guard; per-phase timers; JSONL + TensorBoard metrics; no per-step tensor printing (#11).
"""
from __future__ import annotations

import faulthandler
import os
import sys
import time
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np
import torch

from ..config import Config
from ..data.fewrel import FewRelDataset
from ..data.sampler import EpisodeSampler
from ..models.induction import InductionNetwork
from ..models import reference as ref
from ..ops.optim import FlatParams, FusedOptimizer, lr_at
from ..parallel.dp import DistContext
from . import checkpoint as ckpt
from .metrics import MetricsLogger
from .tb_graph import meta_graph, model_graph


class _HostEpisodes:
    """CPU path: host sampler producing instance indices (same contract as the device sampler)."""

    def __init__(self, data: FewRelDataset, seed: int, nota_rate: float, encoder: str = "bilstm"):
        self.data = data
        self.s = EpisodeSampler(data, seed=seed, nota_rate=nota_rate)
        if encoder == "bert":
            if data.bert is None:
                raise ValueError("dataset has no BERT features (data/bert_tokenize.py)")
            self.arrays = tuple(torch.as_tensor(data.bert[k]) for k in ("ids", "mask", "e1", "e2"))
        else:
            self.arrays = tuple(torch.as_tensor(a) for a in (data.data_word, data.data_pos1, data.data_pos2,
                                                              data.data_mask))

    def sample(self, B, N, K, Q):
        idx, lab = self.s.next_batch_indices(B, N, K, Q)
        return torch.as_tensor(idx.astype(np.int32)), torch.as_tensor(lab.astype(np.int32))

    def state_dict(self):
        return {"bitgen": self.s.rng.bit_generator.state}

    def load_state_dict(self, d):
        self.s.rng.bit_generator.state = d["bitgen"]


class Trainer:
    def __init__(self, cfg: Config, train_data: FewRelDataset, val_data: Optional[FewRelDataset] = None,
                 device: str = "auto", dist_ctx: Optional[DistContext] = None, log: bool = True,
                 test_data: Optional[FewRelDataset] = None):
        cfg.validate()
        self.cfg = cfg
        if cfg.deterministic:
            from ..utils import make_deterministic
            make_deterministic(cfg.seed, trained_word_table=(cfg.train_word_embedding
                                                             or train_data.word_vec_mat is None))
        self.dist = dist_ctx or DistContext.from_env(device if device != "auto" else cfg.device)
        if device not in ("auto", None) and self.dist.world == 1 and torch.device(device).type != self.dist.device.type:
            self.dist.device = torch.device(device)   # (keeps from_env's device index for a matching type)
        self.device = self.dist.device
        self.train_data = train_data
        self.val_data = val_data if val_data is not None else train_data
        self.test_data = test_data
        if cfg.encoder == "bert":
            from ..data.bert_tokenize import synthetic_features
            ds = [self.train_data, self.val_data] + ([test_data] if test_data is not None else [])
            for d in {id(x): x for x in ds}.values():
                if d.bert is None:   # e.g. synthetic data: fold its word ids into the BERT vocabulary
                    d.bert = synthetic_features(d, cfg.bert_vocab, cfg.bert_max_length)
        wv = train_data.word_vec_mat
        vocab = None if wv is not None else int(max(train_data.data_word.max(), 1) + 1)
        self.model = InductionNetwork(cfg, wv, vocab_size=vocab, seed=cfg.seed).to(self.device)
        self.flat = FlatParams(self.model.params.trainable())
        self.grad_views = {n: self.flat.view(self.flat.grad, n) for n in self.flat.names}
        self.glue = None   # fused step plumbing (ops/glue.py): GPU BiLSTM path, BERT gradient slabs
        if self.device.type == "cuda" and cfg.step_glue:
            from ..ops.glue import StepGlue
            self.glue = StepGlue(self.flat)
        if self.dist.initialized:
            self.dist.broadcast_(self.flat.flat, 0)
        l2_names = [n for n, p in self.model.params.trainable().items()
                    if any(p is q for q in self.model.params.l2_vars())]
        self.opt = FusedOptimizer(self.flat, cfg.optimizer, cfg.adam_beta1, cfg.adam_beta2, cfg.adam_eps,
                                  cfg.adagrad_init_acc, l2=cfg.l2_lambda if cfg.use_l2 else 0.0,
                                  l2_mask=self.flat.l2_mask(l2_names) if cfg.use_l2 else None)
        self.global_step = 0
        self.best_acc = 0.0
        rank_seed = cfg.seed * 1009 + 7919 * self.dist.rank
        self.train_eps = self._make_sampler(train_data, rank_seed, cfg.nota_rate)
        self.eval_nota = cfg.nota_rate if cfg.eval_nota_rate < 0 else cfg.eval_nota_rate
        self.val_eps = self._make_sampler(self.val_data, rank_seed + 1, self.eval_nota)
        self.nota_threshold: Optional[float] = cfg.nota_threshold if cfg.nota_threshold >= 0 else None
        self.log = MetricsLogger(cfg.model_dir, enabled=log and self.dist.is_main)
        # the model graph for TensorBoard (the reference's FileWriter(..., sess.graph), model/base.py:125)
        self.log.graph(model_graph(self.model, cfg.N, cfg.K, cfg.Q))
        self.timers = {"sample": 0.0, "fwd_bwd": 0.0, "allreduce": 0.0, "optim": 0.0}   # host (launch) time
        self.gpu_phase_ms = {k: 0.0 for k in self.timers}                                # HIP-event time
        self._pending_events = []
        self._graph = None   # runtime/graph.py::GraphedTrainStep when cfg.use_hip_graph
        self._head_span = self._contiguous_span(("W_s", "M", "ntn_w", "ntn_b"))
        # fault injection (tests / chaos runs): raise at a given global step on a given rank
        self._fault_step = int(os.environ.get("INA_FAULT_STEP", "-1"))
        self._fault_rank = int(os.environ.get("INA_FAULT_RANK", "0"))
        if cfg.resume:
            self.maybe_resume()

    # ------------------------------------------------------------------ plumbing
    def _make_sampler(self, data: FewRelDataset, seed: int, nota: float):
        if self.device.type == "cuda":
            from ..ops.sampler import DeviceDataset, DeviceEpisodeSampler
            dd = DeviceDataset(data, self.device)
            s = DeviceEpisodeSampler(dd, seed=seed, nota_rate=nota)
            s.arrays = dd.arrays(self.cfg.encoder)
            return s
        return _HostEpisodes(data, seed, nota, self.cfg.encoder)

    def _contiguous_span(self, names):
        """(offset, numel) of parameters that are adjacent in the flat buffer, else None."""
        idx = sorted(self.flat.names.index(n) for n in names if n in self.flat.names)
        if not idx or idx != list(range(idx[0], idx[0] + len(idx))):
            return None
        off = self.flat.offsets[idx[0]]
        return off, self.flat.offsets[idx[-1]] + self.flat.numels[idx[-1]] - off

    def _sync(self):
        """Phase boundary: with ``profile`` on a GPU, record a HIP event (no host synchronisation)."""
        if self.device.type == "cuda" and self.cfg.profile:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return None

    def drain_phase_events(self) -> dict:
        """Accumulate the recorded phase events into ``gpu_phase_ms`` (call at a sync point)."""
        for evs in self._pending_events:
            if any(e is None for e in evs):
                continue
            evs[-1].synchronize()
            for k, a, b in zip(("sample", "fwd_bwd", "allreduce", "optim"), evs[:-1], evs[1:]):
                self.gpu_phase_ms[k] += a.elapsed_time(b)
        self._pending_events = []
        return dict(self.gpu_phase_ms)

    def gradient_norms(self, per_variable: bool = False) -> "OrderedDict[str, float]":
        """optimize_loss's gradient summaries from the flat gradient of the last step (read at log points
        only): ``global_norm/gradient_norm`` (one device reduction) and, with ``per_variable``,
        ``gradient_norm/<TF variable name>`` (one segmented reduction).  Under DP the buffer holds the
        all-reduced SUM; the norms are of the applied (1/world-scaled) gradient."""
        g = self.flat.grad.detach().float()
        scale = 1.0 / self.dist.world
        out = OrderedDict()
        sq = g * g
        if per_variable:
            lens = torch.tensor(self.flat.numels, device=g.device)
            seg = torch.segment_reduce(sq, "sum", lengths=lens)
            vals = (seg.sqrt() * scale).tolist()
            out["global_norm/gradient_norm"] = float(sum(v * v for v in vals)) ** 0.5
            for n, v in zip(self.flat.names, vals):
                out["gradient_norm/" + self.model.params.tf_name(n)] = v
        else:
            out["global_norm/gradient_norm"] = float(sq.sum().sqrt()) * scale
        return out

    @property
    def graph_step_enabled(self) -> bool:
        """The train step runs as a captured hipGraph: ``use_hip_graph``, or automatically for small
        (launch-bound) steps of the fused BiLSTM path."""
        cfg = self.cfg
        if self.device.type != "cuda" or cfg.encoder != "bilstm" or self.glue is None:
            return False
        # only the fused BiLSTM kernels read the dropout seed from device memory (seed_dev); the wide /
        # per-step paths take it as a host int that a captured graph would freeze (same mask every replay)
        if not self.model.use_fused_lstm(cfg.max_length):
            return False
        return cfg.use_hip_graph or 0 < cfg.episodes_per_step <= cfg.hip_graph_max_episodes

    @property
    def skipped_steps(self) -> int:
        """Optimizer steps skipped by the NaN/Inf guard (synchronises on the GPU)."""
        return self.opt.skipped()

    def dropout_seed(self) -> int:
        return (self.cfg.seed * 2654435761 + self.global_step * 97 + self.dist.rank * 7919) & 0x7FFFFFFF

    # ------------------------------------------------------------------ steps
    def train_step(self) -> Tuple[float, float]:
        """One optimiser step; returns host floats (synchronises)."""
        loss, acc = self.train_step_async()
        return float(loss), float(acc)

    def train_step_async(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """One optimiser step with NO host synchronisation; returns device (loss, acc) tensors.

        Gradients are written by the fused backward functions straight into the flat gradient
        buffer (grad_views), which is also the DP all-reduce bucket and the fused optimizer input."""
        cfg = self.cfg
        B, N, K, Q = cfg.episodes_per_step, cfg.N, cfg.K, cfg.Q
        if self.graph_step_enabled and self.global_step != self._fault_step:
            if self._graph is None:
                from .graph import GraphedTrainStep
                self._graph = GraphedTrainStep(self)   # first step eager (warm-up) + capture, then replays
            self._last_lr = lr_at(self.global_step, cfg.learning_rate, cfg.decay_steps, cfg.decay_rate,
                                  cfg.staircase, cfg.lr_schedule)
            return self._graph.step()
        if self.global_step == self._fault_step and self.dist.rank == self._fault_rank:
            raise RuntimeError(f"injected fault at step {self.global_step} on rank {self.dist.rank} (INA_FAULT_STEP)")
        t0 = time.perf_counter()
        e0 = self._sync()
        idx, labels = self.train_eps.sample(B, N, K, Q)
        e1 = self._sync()
        t1 = time.perf_counter()
        self.flat.zero_grad()
        gv = self.grad_views if self.device.type == "cuda" else None
        ov = None
        if self.dist.initialized and cfg.encoder == "bert" and self.device.type == "cuda":
            # per-layer buckets all-reduced under the rest of backward (~28 MB fp32 each at BERT-base)
            from ..ops.bert import layer_spans
            ov = self.dist.overlap(self.flat.grad, layer_spans(self.model, self.flat.names, self.flat.offsets,
                                                               self.flat.numels))
        elif self.dist.initialized and self.glue is not None and self._head_span is not None:
            # BiLSTM step: the relation head's gradients (W_s, M, w, b: ~94% of the parameters) are final
            # after the head backward -> their all-reduce runs under the attention + BiLSTM backward
            ov = self.dist.overlap(self.flat.grad, [self._head_span])
        loss, acc_t, _ = self.model.forward_train(idx.view(-1), self.train_eps.arrays, B, N, K, Q, labels,
                                                  dropout_seed=self.dropout_seed(), grad_views=gv, overlap=ov,
                                                  glue=self.glue)
        torch.autograd.backward(loss, self.glue.one if self.glue is not None else None)
        if self.glue is not None:
            self.glue.flush()
        self.flat.sync_grads_into_flat()
        e2 = self._sync()
        t2 = time.perf_counter()
        if ov is not None:
            ov.finish()
        elif self.dist.initialized:
            self.dist.allreduce_buckets_(self.flat.grad)
        e3 = self._sync()
        t3 = time.perf_counter()
        lr = lr_at(self.global_step, cfg.learning_rate, cfg.decay_steps, cfg.decay_rate, cfg.staircase,
                   cfg.lr_schedule)
        # NaN/Inf guard: the update is skipped on the device when a gradient / the loss is not finite
        # (DP: only the all-reduced gradients are checked, so every rank takes the same decision)
        self.opt.step(lr, grad_scale=1.0 / self.dist.world, check_finite=cfg.grad_check_finite,
                      loss=loss if self.dist.world == 1 else None)
        self.global_step += 1
        e4 = self._sync()
        if e0 is not None:
            self._pending_events.append((e0, e1, e2, e3, e4))
        t4 = time.perf_counter()
        self.timers["sample"] += t1 - t0
        self.timers["fwd_bwd"] += t2 - t1
        self.timers["allreduce"] += t3 - t2
        self.timers["optim"] += t4 - t3
        self._last_lr = lr
        return loss.detach(), acc_t

    @torch.no_grad()
    def evaluate(self, iters: int, N: Optional[int] = None, K: Optional[int] = None, Q: Optional[int] = None,
                 batch: Optional[int] = None, sampler=None, nota_threshold: Optional[float] = None) -> float:
        """Mean over episodes of per-episode accuracy (model/base.py:186-208), mask fed (fix #1)."""
        cfg = self.cfg
        N, K, Q = N or cfg.eN, K or cfg.eK, Q or cfg.eQ
        B = batch or cfg.eval_batch or max(1, min(cfg.episodes_per_step, iters))
        s = sampler or self.val_eps
        if nota_threshold is None:
            nota_threshold = self.nota_threshold
        done, acc_sum = 0, 0.0
        while done < iters:
            b = min(B, iters - done)
            idx, labels = s.sample(b, N, K, Q)
            probs, _ = self.model(idx.view(-1), s.arrays, b, N, K, Q, training=False)
            pred = ref.predict(probs, nota_threshold)
            acc_sum += float((pred == labels.long()).float().mean(-1).sum())
            done += b
        acc = acc_sum / max(1, done)
        return self.dist.mean_scalars([acc])[0]

    # ------------------------------------------------------------------ loop
    def train(self) -> float:
        cfg = self.cfg
        self.log.print(f"{cfg.N}-way-{cfg.K}-shot Few-Shot Relation Classification")
        self.log.print(f"Model: {cfg.model_name}  world={self.dist.world}  device={self.device}  "
                       f"episodes/step/rank={cfg.episodes_per_step}")
        it_loss = it_acc = it_n = 0.0
        start = self.global_step
        t_start = time.time()
        pend_loss = pend_acc = None
        pend_n = 0
        seen_skips = self.skipped_steps if cfg.grad_check_finite else 0
        if cfg.watchdog_s > 0:
            self.log.print(f"watchdog: abort if a step exceeds {cfg.watchdog_s:.0f}s")
        for it in range(start, cfg.train_iter):
            if cfg.watchdog_s > 0:   # hung collective / kernel -> traceback + exit (launcher restarts, resume)
                faulthandler.dump_traceback_later(cfg.watchdog_s, repeat=False, file=sys.stderr, exit=True)
            loss_t, acc_t = self.train_step_async()
            if cfg.save_every > 0 and self.global_step % cfg.save_every == 0:
                self.save()
            # accumulate on device; the host only synchronises at log / reset / eval points.  The first
            # term is cloned: with use_hip_graph loss_t/acc_t are the graph's static outputs, which the
            # next replay overwrites
            pend_loss = loss_t.clone() if pend_loss is None else pend_loss + loss_t
            pend_acc = acc_t.clone() if pend_acc is None else pend_acc + acc_t
            pend_n += 1
            if (it % cfg.log_every == 0 or it % cfg.val_step == 0 or (it + 1) % cfg.val_step == 0
                    or it + 1 == cfg.train_iter):
                pl, pa = float(pend_loss), float(pend_acc)
                if hasattr(self.train_eps, "check"):
                    self.train_eps.check()   # device sampler's rejection-limit flag
                if cfg.grad_check_finite:
                    sk = self.skipped_steps
                    if sk > seen_skips:
                        self.log.print(f"[warn] {sk - seen_skips} step(s) with non-finite gradients/loss up to step "
                                       f"{it + 1}: update skipped (parameters and optimizer moments unchanged)")
                        seen_skips = sk
                it_loss += pl
                it_acc += pa
                it_n += pend_n
                pend_loss = pend_acc = None
                pend_n = 0
                summ = set(x.strip() for x in cfg.summaries.split(",") if x.strip())
                norms = (self.gradient_norms("gradient_norm" in summ)
                         if summ & {"global_gradient_norm", "gradient_norm"} else {})
                if "global_gradient_norm" not in summ:
                    norms.pop("global_norm/gradient_norm", None)
                self.log.log(self.global_step, "train", loss=it_loss / it_n, accuracy=it_acc / it_n,
                             learning_rate=self._last_lr, **norms)
                if cfg.profile and self.device.type == "cuda":
                    self.log.log(self.global_step, "profile", **{f"gpu_{k}_ms": v for k, v in
                                                                 self.drain_phase_events().items()},
                                 **{f"host_{k}_s": v for k, v in self.timers.items()})
            if it % cfg.log_every == 0:
                el = time.time() - t_start
                eps = (it - start + 1) * cfg.episodes_per_step * self.dist.world / max(el, 1e-9)
                self.log.print(f"[train] step:{it + 1:4} | loss: {it_loss / it_n:2.6f}, accuracy: "
                               f"{100 * it_acc / it_n:3.2f}% | {eps:.1f} episodes/s")
                self.log.flush()
            if it % cfg.val_step == 0:
                it_loss = it_acc = it_n = 0.0
            if (it + 1) % cfg.val_step == 0:
                if cfg.watchdog_s > 0:
                    faulthandler.cancel_dump_traceback_later()   # evaluation is not a train step
                acc_val = self.evaluate(cfg.val_iter)
                self.log.log(self.global_step, "val", accuracy=acc_val)
                self.log.print(f"[EVAL] step {it + 1} accuracy: {100 * acc_val:.2f}%")
                if acc_val > self.best_acc:
                    self.best_acc = acc_val
                    self.log.print(f"Best checkpoint.[EVAL] accuracy :{acc_val}")
                    self.save(best=True)
        if cfg.watchdog_s > 0:
            faulthandler.cancel_dump_traceback_later()
        self.log.print("\n####################\n")
        self.log.print("Finish training :" + cfg.ckpt_name)
        if cfg.test_best and self.best_acc > 0.0:
            best = ckpt.best(cfg.model_dir)   # the best-val pointer, not the newest (periodic) checkpoint
            if best is not None:
                step = self.global_step
                self.load(best)
                self.log.print(f"test from best checkpoint {best} (val acc {self.best_acc:.4f}; trained {step} steps)")
        if self.eval_nota > 0.0 and self.nota_threshold is None:
            from .evaluate import collect_probs, select_nota_threshold
            tp, tl = collect_probs(self, self.val_eps, min(cfg.val_iter, 1000), cfg.eN, cfg.eK, cfg.eQ,
                                   cfg.eval_batch or None)
            self.nota_threshold = select_nota_threshold(tp, tl, cfg.eN)
            self.log.print(f"NOTA threshold (tuned on val): {self.nota_threshold:.2f}")
        if self.test_data is not None:   # e.g. another domain (FewRel 2.0 DA) or a held-out split
            from .evaluate import evaluate_dataset
            rep = evaluate_dataset(self, self.test_data, cfg.test_iter, cfg.eN, cfg.eK, cfg.eQ, self.eval_nota,
                                   self.nota_threshold, cfg.eval_batch or None)
            test_acc = rep.accuracy
            self.log.log(self.global_step, "test", **{k: v for k, v in rep.to_dict().items()
                                                      if isinstance(v, float) and v == v})
        else:
            test_acc = self.evaluate(cfg.test_iter)
            self.log.log(self.global_step, "test", accuracy=test_acc)
        self.log.print(f"Test accuracy: {test_acc}")
        self.log.close()
        return test_acc

    # ------------------------------------------------------------------ checkpoint
    def state_tensors(self) -> "OrderedDict[str, torch.Tensor]":
        p = self.model.params
        out = OrderedDict(p.tf_state())
        names = list(self.flat.names)
        st = self.opt.state_tensors()
        for i, attr in enumerate(names):
            tf = p.tf_name(attr)
            if self.opt.kind == "adam":
                out[tf + "/Adam"] = self.flat.view(st["m"], attr)
                out[tf + "/Adam_1"] = self.flat.view(st["v"], attr)
            else:
                out[tf + "/Adagrad"] = self.flat.view(st["acc"], attr)
        if self.opt.kind == "adam":
            out["beta1_power"] = torch.tensor(self.cfg.adam_beta1 ** (self.opt.t + 1), dtype=torch.float32)
            out["beta2_power"] = torch.tensor(self.cfg.adam_beta2 ** (self.opt.t + 1), dtype=torch.float32)
        out["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return out

    def save(self, best: bool = False) -> Optional[str]:
        """Collective under DP (every rank calls it at the same step): each rank's own sampler state is
        gathered, then rank 0 writes.  ``best``: this is the best-val checkpoint (``test_best``)."""
        samplers = self.dist.all_gather_objects(self.train_eps.state_dict())
        skipped = self.skipped_steps
        if not self.dist.is_main:
            return None
        meta = {"best_acc": self.best_acc, "optimizer_t": self.opt.t, "optimizer_t_counts": "applied",
                "config": self.cfg.to_dict(),
                "train_samplers": samplers, "skipped_steps": skipped, "world_size": self.dist.world}
        mg = None
        if self.cfg.tf_checkpoint:
            if getattr(self, "_meta_graph", None) is None:   # built once (the graph does not change)
                self._meta_graph = meta_graph(self.model, self.cfg.N, self.cfg.K, self.cfg.Q, self.cfg.max_to_keep)
            mg = self._meta_graph
        return ckpt.save(self.cfg.model_dir, self.cfg.ckpt_name, self.global_step, self.state_tensors(), meta,
                         self.cfg.max_to_keep, best=best, tf_format=self.cfg.tf_checkpoint, meta_graph=mg)

    def load(self, stem: str, prefer: str = "safetensors") -> None:
        """Restore from ``stem`` (either checkpoint format; ``prefer="tf"``: the TF bundle copy)."""
        tensors, meta = ckpt.load(stem, prefer)
        p = self.model.params
        p.load_tf_state(tensors, strict=False)
        st = self.opt.state_tensors()
        with torch.no_grad():
            for attr in self.flat.names:
                tf = p.tf_name(attr)
                if self.opt.kind == "adam" and tf + "/Adam" in tensors:
                    self.flat.view(st["m"], attr).copy_(tensors[tf + "/Adam"])
                    self.flat.view(st["v"], attr).copy_(tensors[tf + "/Adam_1"])
                elif self.opt.kind == "adagrad" and tf + "/Adagrad" in tensors:
                    self.flat.view(st["acc"], attr).copy_(tensors[tf + "/Adagrad"])
        self.global_step = int(tensors["global_step"].item()) if "global_step" in tensors else int(meta["global_step"])
        self.best_acc = float(meta.get("best_acc", 0.0))
        skipped = int(meta.get("skipped_steps", 0))
        # optimizer_t: applied Adam updates (older checkpoints stored the step count, skips included)
        if "optimizer_t" in meta:
            t = int(meta["optimizer_t"])
            if meta.get("optimizer_t_counts") != "applied":   # older checkpoints counted the skipped steps too
                t -= skipped
        else:
            t = self.global_step - skipped
        self.opt.load_counters(max(0, t), skipped)
        self._restore_sampler(meta)
        if self.dist.initialized:
            self.dist.broadcast_(self.flat.flat, 0)

    def _restore_sampler(self, meta: dict) -> None:
        """Each rank restores ITS OWN sampler state (rank-folded seed), so the DP ranks keep drawing
        different episodes after a restart.  With a different world size the per-rank streams do not
        map onto the new ranks: keep the fresh rank-folded seeds and only carry the call counter of the
        device sampler forward (new episodes, no replay of the pre-restart ones)."""
        states = meta.get("train_samplers")
        if states is None:   # older single-state checkpoints: rank 0's state; exact only at world size 1
            states = [meta["train_sampler"]] if "train_sampler" in meta else []
            same_world = bool(states) and int(meta.get("world_size", 1)) == 1 and self.dist.world == 1
        else:
            same_world = len(states) == self.dist.world
        if same_world:
            self.train_eps.load_state_dict(states[self.dist.rank])
        elif states and "calls" in states[0] and hasattr(self.train_eps, "calls"):
            self.train_eps.calls = int(states[0]["calls"])

    def maybe_resume(self) -> bool:
        stem = ckpt.latest(self.cfg.model_dir)
        if stem is None:
            return False
        self.load(stem)
        self.log.print(f"resumed from {stem} at step {self.global_step}")
        return True
