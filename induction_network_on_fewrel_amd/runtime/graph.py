"""HIP-graph capture of the BiLSTM training step (``Config.use_hip_graph``).

One optimiser step of the default model is ~50 kernels (sampling, packs, BiLSTM, attention,
routing, NTN, loss, slab reductions, Adam); replaying them as one hipGraph removes the per-launch
host cost that otherwise leaves the GPU idle between small kernels.

A captured graph replays fixed kernel arguments, so every per-step scalar lives in device memory:
``ina.step_control`` (the graph's first node) computes the dropout seed, the sampler seed and the
(bias-corrected) learning rate from device counters, with the same formulas as the eager path
(``Trainer.dropout_seed``, ``DeviceEpisodeSampler.sample``, ``ops/optim.py::lr_at`` + TF1 Adam),
and advances the counters.  The host mirrors the counters (global_step, optimizer t, sampler calls)
so checkpoints and logging are unchanged.

world_size > 1: the graph covers sampling + forward + backward; the RCCL bucket all-reduce and the
fused optimizer (reading the device learning rate) run eagerly after each replay.
"""
from __future__ import annotations

import torch

from ..ops._ext import ops


class GraphedTrainStep:
    def __init__(self, trainer):
        self.tr = trainer
        cfg = trainer.cfg
        dev = trainer.device
        self.dist = trainer.dist
        self.with_opt = trainer.dist.world == 1
        # ctl: [dropout seed, sampler seed, global step, sampler calls, optimizer step calls (t_base + calls;
        # the Adam kernel subtracts the device skip count)]
        s = trainer.train_eps
        self.ctl = torch.tensor([0, 0, trainer.global_step, s.calls, trainer.opt.t_host, 0, 0, 0], dtype=torch.int32,
                                device=dev)
        self.lrt = torch.zeros(2, dtype=torch.float32, device=dev)
        self.seedA = (cfg.seed * 2654435761 + trainer.dist.rank * 7919) & 0x7FFFFFFF
        self.seedB = s.seed_base()
        self.graph = None
        self.loss = self.acc = None

    def _capture(self):
        """First call: one real (eager) step on a side stream (allocator warm-up), then capture."""
        tr = self.tr
        dev = tr.device
        s = tr.train_eps
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            loss, acc = self._body()
            self._after_eager_or_replay()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        saved = (s.calls, tr.opt.calls)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss, self.acc = self._body()
        s.calls, tr.opt.calls = saved           # capture does not execute: undo the host bookkeeping
        return loss, acc

    def _body(self):
        tr, cfg = self.tr, self.tr.cfg
        B, N, K, Q = cfg.episodes_per_step, cfg.N, cfg.K, cfg.Q
        o = ops()
        o.step_control(self.ctl, self.lrt, self.seedA, self.seedB, cfg.learning_rate, float(cfg.decay_steps),
                       cfg.decay_rate, bool(cfg.staircase), cfg.lr_schedule == "constant", tr.opt.kind == "adam",
                       cfg.adam_beta1, cfg.adam_beta2)
        idx, labels = tr.train_eps.sample(B, N, K, Q, seed_dev=self.ctl[1:2])
        tr.flat.zero_grad()
        loss, acc, _ = tr.model.forward_train(idx.view(-1), tr.train_eps.arrays, B, N, K, Q, labels, dropout_seed=0,
                                              grad_views=tr.grad_views, seed_dev=self.ctl[0:1], glue=tr.glue)
        torch.autograd.backward(loss, tr.glue.one if tr.glue is not None else None)
        if tr.glue is not None:
            tr.glue.flush()
        tr.flat.sync_grads_into_flat()
        if self.with_opt:
            tr.opt.step(0.0, grad_scale=1.0, lr_dev=self.lrt[0:1], check_finite=cfg.grad_check_finite, loss=loss,
                        t_dev=self.ctl[4:5])
        return loss.detach(), acc

    def _after_eager_or_replay(self):
        tr = self.tr
        if not self.with_opt:
            tr.dist.allreduce_buckets_(tr.flat.grad)
            tr.opt.step(0.0, grad_scale=1.0 / tr.dist.world, lr_dev=self.lrt[0:1], check_finite=tr.cfg.grad_check_finite,
                        t_dev=self.ctl[4:5])
        tr.global_step += 1

    def step(self):
        """One training step: the first call runs it eagerly and captures; later calls replay.
        Returns the step's device (loss, acc) (graph outputs stay valid until the next replay)."""
        tr = self.tr
        if self.graph is None:
            return self._capture()
        self.graph.replay()
        tr.train_eps.calls += 1
        if self.with_opt:
            tr.opt.calls += 1
        self._after_eager_or_replay()
        return self.loss, self.acc
