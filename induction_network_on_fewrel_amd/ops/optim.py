"""Flat-buffer parameter store + fused optimizers (K10 of SURVEY 2.3).

All trainable tensors are views into ONE contiguous fp32 buffer and their ``.grad`` are views into
ONE contiguous fp32 gradient buffer. That single gradient buffer is the data-parallel all-reduce
bucket (parallel/dp.py) and the fused optimizer updates the whole model with one kernel.

Reference: model/base.py:94-99 -- ``tf.train.exponential_decay(1e-3, step, 100, 0.9, staircase=True)``
+ ``optimize_loss(..., optimizer="Adam")`` (TF1 Adam defaults, no clipping).
On CPU the same math runs in torch (plumbing path, BASELINE config 1).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, Optional

import torch
from torch import nn

from ._ext import ops


def lr_at(step: int, base: float, decay_steps: int, decay_rate: float, staircase: bool = True,
          schedule: str = "exponential") -> float:
    """tf.train.exponential_decay evaluated at ``global_step = step`` (before the increment)."""
    if schedule == "constant":
        return base
    p = step / decay_steps
    if staircase:
        p = math.floor(p)
    return base * decay_rate ** p


class FlatParams:
    """Re-homes the given parameters into one flat buffer (params and grads)."""

    def __init__(self, named: "OrderedDict[str, nn.Parameter]"):
        self.names = list(named.keys())
        self.params = list(named.values())
        self.shapes = [tuple(p.shape) for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.numel = off
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        # gradient storage = [grad (numel) | pad | NaN/Inf guard flag]: zero_grad clears the flag with the
        # gradients in one fill (the flag word sits 16-B aligned behind the last gradient)
        self._gstore = torch.zeros(self.numel + 8 - self.numel % 4, dtype=torch.float32, device=dev)
        self.grad = self._gstore[:self.numel]
        self.guard = self._gstore[-1:]
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + n].view(p.shape)
                p.grad = self.grad[o:o + n].view(p.shape)

    def view(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        i = self.names.index(name)
        return buf[self.offsets[i]:self.offsets[i] + self.numels[i]].view(self.shapes[i])

    def zero_grad(self) -> None:
        self._gstore.zero_()
        # autograd may have replaced .grad with a fresh tensor (e.g. when a grad was None); re-home
        for p, o, n in zip(self.params, self.offsets, self.numels):
            g = p.grad
            if g is None or g.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view(p.shape)

    def sync_grads_into_flat(self) -> None:
        """Copy any grad that autograd stored outside the flat buffer back into it."""
        for p, o, n in zip(self.params, self.offsets, self.numels):
            g = p.grad
            if g is not None and g.data_ptr() != self.grad[o:o + n].data_ptr():
                self.grad[o:o + n].copy_(g.reshape(-1))
                p.grad = self.grad[o:o + n].view(p.shape)

    def l2_mask(self, names) -> torch.Tensor:
        m = torch.zeros(self.numel, dtype=torch.uint8, device=self.flat.device)
        for nm in names:
            i = self.names.index(nm)
            m[self.offsets[i]:self.offsets[i] + self.numels[i]] = 1
        return m


class FusedOptimizer:
    """Adam (TF1 form) or Adagrad over a FlatParams store; GPU -> one HIP kernel, CPU -> torch."""

    def __init__(self, flat: FlatParams, kind: str = "adam", beta1: float = 0.9, beta2: float = 0.999,
                 eps: float = 1e-8, adagrad_init: float = 0.1, l2: float = 0.0,
                 l2_mask: Optional[torch.Tensor] = None):
        self.flat = flat
        self.kind = kind
        self.b1, self.b2, self.eps = beta1, beta2, eps
        self.l2 = float(l2)
        self.l2_mask = l2_mask if (l2_mask is not None and self.l2 > 0) else None
        # Adam's t counts APPLIED updates only (a step the NaN/Inf guard skips must not advance the bias
        # correction): t = t_base + calls - skips since the base, where the base is set at construction /
        # checkpoint load.  On the GPU the kernel derives t from the host call count (or the graph's
        # device counter) minus the device skip counter, so no host synchronisation is needed.
        self.t_base = 0       # applied updates at the base
        self.calls = 0        # step() calls since the base (applied + skipped)
        dev = flat.flat.device
        self.skips_base = 0   # skipped steps before the base (restored from a checkpoint)
        self.skips_cpu = 0    # CPU path: skipped steps since the base
        self.skips_dev = torch.zeros(1, dtype=torch.int32, device=dev) if dev.type == "cuda" else None
        if kind == "adam":
            self.m = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
            self.v = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        elif kind == "adagrad":
            self.acc = torch.full((flat.numel,), adagrad_init, dtype=torch.float32, device=dev)
        else:
            raise ValueError(kind)

    def state_tensors(self) -> Dict[str, torch.Tensor]:
        if self.kind == "adam":
            return {"m": self.m, "v": self.v}
        return {"acc": self.acc}

    def _skips_since_base(self) -> int:
        return self.skips_cpu + (int(self.skips_dev.item()) if self.skips_dev is not None else 0)

    def skipped(self) -> int:
        """Steps the NaN/Inf guard skipped so far (reads the device counter: synchronises)."""
        return self.skips_base + self._skips_since_base()

    @property
    def t(self) -> int:
        """Applied Adam updates (TF's beta powers are beta^(t+1) after them); synchronises on the GPU."""
        return self.t_base + self.calls - self._skips_since_base()

    @property
    def t_host(self) -> int:
        """What the kernel subtracts the device skip count from: t_base + calls (no synchronisation)."""
        return self.t_base + self.calls

    def load_counters(self, t_applied: int, skipped_total: int) -> None:
        """Re-base the step accounting (checkpoint restore)."""
        self.t_base, self.calls = int(t_applied), 0
        self.skips_base, self.skips_cpu = int(skipped_total), 0
        if self.skips_dev is not None:
            self.skips_dev.zero_()

    def step(self, lr: float, grad_scale: float = 1.0, lr_dev: Optional[torch.Tensor] = None,
             check_finite: bool = False, loss: Optional[torch.Tensor] = None,
             t_dev: Optional[torch.Tensor] = None) -> None:
        """``lr``: the scheduled rate; Adam's bias correction is applied for the applied-step count.
        ``lr_dev`` / ``t_dev``: device scalars overriding ``lr`` and the host step count (HIP-graph
        replay: written by ina.step_control inside the captured step).

        ``check_finite``: skip the whole update (parameters and moments untouched) when any gradient
        -- or ``loss``, a scalar -- is NaN/Inf.  On the GPU the decision is made on the device
        (``ina.nonfinite_flag`` -> guard word in the gradient buffer tail -> the optimizer kernel), so
        the step stays asynchronous / graph-capturable; skips are counted in ``skips_dev``.  Under DP
        pass the all-reduced gradients and no loss, so every rank takes the same decision."""
        self.calls += 1
        p, g = self.flat.flat, self.flat.grad
        if p.is_cuda:
            o = ops()
            guard = None
            if check_finite:
                guard = self.flat.guard
                o.nonfinite_flag(g, loss.detach().reshape(1).float() if loss is not None else None, guard)
            if self.kind == "adam":
                o.adam_step(p, self.m, self.v, g, self.l2_mask, lr, self.t_host, self.b1, self.b2, self.eps, grad_scale,
                            self.l2, lr_dev, t_dev, guard, self.skips_dev)
            else:
                o.adagrad_step(p, self.acc, g, self.l2_mask, lr, grad_scale, self.l2, lr_dev, guard, self.skips_dev)
            return
        if check_finite and (not bool(torch.isfinite(g).all())
                             or (loss is not None and not bool(torch.isfinite(loss.detach()).all()))):
            self.skips_cpu += 1
            return
        with torch.no_grad():
            gg = g * grad_scale
            if self.l2_mask is not None:
                gg = gg + self.l2 * p * self.l2_mask.float()
            if self.kind == "adam":
                t = self.t   # applied updates including this one (CPU: no device counter)
                lr_t = lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
                self.m.mul_(self.b1).add_(gg, alpha=1 - self.b1)
                self.v.mul_(self.b2).addcmul_(gg, gg, value=1 - self.b2)
                p.sub_(lr_t * self.m / (self.v.sqrt() + self.eps))
            else:
                self.acc.addcmul_(gg, gg)
                p.sub_(lr * gg / self.acc.sqrt())
