"""Fused optimizer step accounting under the NaN/Inf guard (ops/optim.py, optim.hip::adam_kernel).

A step whose gradient is not finite is skipped on the device: parameters and moments stay unchanged
AND Adam's bias-correction count t does not advance.  So "step 1, NaN step 2, step 3" must leave the
same parameters and moments, bit for bit, as "step 1, step 3" on a run that never saw step 2.
"""
from collections import OrderedDict

import pytest
import torch
from torch import nn

from induction_network_on_fewrel_amd.ops.optim import FlatParams, FusedOptimizer


def _run(device, grads, kind="adam"):
    torch.manual_seed(0)
    named = OrderedDict(a=nn.Parameter(torch.randn(37, 5)), b=nn.Parameter(torch.randn(300)))
    for p in named.values():
        p.data = p.data.to(device)
    flat = FlatParams(named)
    opt = FusedOptimizer(flat, kind)
    for i, g in enumerate(grads):
        flat.zero_grad()
        flat.grad.copy_(g.to(device))
        opt.step(1e-2 * 0.9 ** i, check_finite=True)
    st = {k: v.detach().cpu().clone() for k, v in opt.state_tensors().items()}
    return flat.flat.detach().cpu().clone(), st, opt.t, opt.skipped()


def _grads(n):
    g = torch.Generator().manual_seed(3)
    g1, g3 = torch.randn(n, generator=g), torch.randn(n, generator=g)
    bad = torch.randn(n, generator=g)
    bad[17] = float("nan")
    return g1, bad, g3


def _check(device, kind):
    n = 37 * 5 + 300
    g1, bad, g3 = _grads(n)
    p_skip, st_skip, t_skip, sk = _run(device, [g1, bad, g3], kind)
    # the reference run never sees the bad step; its lr schedule index shifts, so feed the same rates
    torch.manual_seed(0)
    named = OrderedDict(a=nn.Parameter(torch.randn(37, 5)), b=nn.Parameter(torch.randn(300)))
    for p in named.values():
        p.data = p.data.to(device)
    flat = FlatParams(named)
    opt = FusedOptimizer(flat, kind)
    for lr, g in ((1e-2, g1), (1e-2 * 0.9 ** 2, g3)):
        flat.zero_grad()
        flat.grad.copy_(g.to(device))
        opt.step(lr, check_finite=True)
    assert sk == 1 and t_skip == 2 and opt.t == 2
    assert torch.equal(p_skip, flat.flat.detach().cpu())
    for k, v in opt.state_tensors().items():
        assert torch.equal(st_skip[k], v.detach().cpu()), k


@pytest.mark.parametrize("kind", ["adam", "adagrad"])
def test_guard_skip_does_not_advance_adam_t_cpu(kind):
    _check("cpu", kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adam", "adagrad"])
def test_guard_skip_does_not_advance_adam_t_gpu(kind):
    _check("cuda", kind)


def test_load_counters_rebases():
    named = OrderedDict(a=nn.Parameter(torch.zeros(4)))
    opt = FusedOptimizer(FlatParams(named))
    opt.load_counters(7, 2)
    assert opt.t == 7 and opt.skipped() == 2 and opt.t_host == 7
    opt.step(1e-3)
    assert opt.t == 8 and opt.t_host == 8
