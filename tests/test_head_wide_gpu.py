"""Wide induction / relation head (csrc/kernels/head_wide.hip + the GEMMs of ops/wide.py) against the
fp32 oracle (models/reference.py::head_forward, dynamic_routing, mse_loss / ce_loss): the paper's
H = 256 with Q = 20 (N*Q = 100), the reference Base default's H = 200, BERT's H = 768, both relation
heads, 1- and 5-shot."""
import pytest
import torch

from induction_network_on_fewrel_amd.models import reference as ref
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.ops.wide import HeadWideLossFn, head_wide, head_wide_ok

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _nrel(a, b):
    """Norm-relative error.  Gradients are compared with the oracle evaluated at the same bf16-rounded NTN
    operands (reference.head_forward(bf16=True)): against the pure fp32 oracle every bf16 rounding of C, M
    or Q flips the ReLU mask of the few pre-activations within rounding distance of 0, and each flip moves
    a full-size gradient term (~4% norm error at random init) -- a property of bf16 NTN, not of the kernels."""
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _params(H, N, h, head, gen):
    Ws = torch.randn(H, H, generator=gen) * (2.0 / (2 * H)) ** 0.5
    M = torch.randn(H, H, h, generator=gen) * (2.0 / (H + H * h)) ** 0.5 * 4
    if head == "reference":
        w, b = torch.randn(h * N, N, generator=gen) * 0.1, torch.randn(N, generator=gen) * 0.1
    else:
        w, b = torch.randn(h, 1, generator=gen) * 0.1, torch.randn(1, generator=gen) * 0.1
    return {k: v.to(DEV).requires_grad_(True) for k, v in
            dict(W_s=Ws, M=M, ntn_w=w, ntn_b=b).items()}


@pytest.mark.parametrize("H,N,K,Q", [(256, 5, 5, 20), (256, 5, 1, 20), (200, 5, 5, 5), (768, 10, 5, 5)])
@pytest.mark.parametrize("head", ["reference", "paper"])
def test_wide_head_probs_and_grads(H, N, K, Q, head):
    E, h, R = 6, 100, 3
    assert head_wide_ok(H, N, K, R, head)
    gen = torch.Generator().manual_seed(H + N * K + Q)
    p = _params(H, N, h, head, gen)
    e = (torch.randn(E * (N * K + N * Q), H, generator=gen) * 0.3).to(DEV).requires_grad_(True)
    probs = head_wide(e, p, E, N, K, Q, R, head)
    gout = torch.randn(probs.shape, generator=gen).to(DEV)
    (probs * gout).sum().backward()
    got = {k: v.grad.clone() for k, v in p.items()}
    ge = e.grad.clone()
    for v in list(p.values()) + [e]:
        v.grad = None
    with torch.no_grad():
        assert _relerr(probs, ref.head_forward(p, e, E, N, K, Q, R, head)) < 2e-2   # vs the fp32 oracle
    pr = ref.head_forward(p, e, E, N, K, Q, R, head, bf16=True)
    (pr * gout).sum().backward()
    assert _relerr(probs.detach(), pr.detach()) < 5e-3
    assert _nrel(ge, e.grad) < 2e-2
    for k in p:   # paper head + CE: the shared bias cancels in the softmax (its exact gradient is 0)
        assert _nrel(got[k], p[k].grad) < 2e-2 or float((got[k] - p[k].grad).abs().max()) < 1e-5, k


@pytest.mark.parametrize("H,K,R", [(256, 5, 3), (200, 1, 3), (256, 20, 5), (768, 5, 2)])
def test_routing_wide_kernels_fp32_exact(H, K, R):
    """routing_wide_fwd / _bwd are fp32 end to end: tight tolerance against the oracle from e_hat."""
    o = ops()
    items = 37
    gen = torch.Generator().manual_seed(K * R + H)
    eh = (torch.randn(items * K, H, generator=gen) * 0.2).to(DEV)
    cls, cls_bf = o.routing_wide_fwd(eh, items, K, R)
    x = eh.view(items, 1, K, H).clone().requires_grad_(True)
    c = ref.dynamic_routing(x, torch.eye(H, device=DEV), R).view(items, H)
    assert _relerr(cls, c.detach()) < 1e-5
    assert torch.equal(cls_bf, cls.to(torch.bfloat16))
    dc = torch.randn(items, H, generator=gen).to(DEV)
    c.backward(dc)
    deh = o.routing_wide_bwd(eh, dc, items, K, R)
    assert _relerr(deh, x.grad.view(items * K, H)) < 1e-4


@pytest.mark.parametrize("loss_type", ["mse", "ce", "ce_nota"])
@pytest.mark.parametrize("head", ["reference", "paper"])
def test_wide_head_loss_node(loss_type, head):
    """HeadWideLossFn (head + ina.head_loss) == oracle head + loss: value, accuracy and gradients (ce_nota: a
    quarter of the queries are NOTA, label N)."""
    E, N, K, Q, H, h, R = 8, 5, 5, 20, 256, 100, 3
    gen = torch.Generator().manual_seed(7)
    p = _params(H, N, h, head, gen)
    e = (torch.randn(E * (N * K + N * Q), H, generator=gen) * 0.3).to(DEV).requires_grad_(True)
    labels = torch.arange(N, device=DEV).repeat_interleave(Q).repeat(E).view(E, N * Q).int()
    if loss_type == "ce_nota":
        labels[:, ::4] = N
    loss, acc, probs = HeadWideLossFn.apply(e, p["W_s"], p["M"], p["ntn_w"], p["ntn_b"], labels,
                                            (E, N, K, Q, R, head == "paper"), loss_type, "mean")
    (loss * 3.0).backward()
    got = {k: v.grad.clone() for k, v in p.items()}
    ge = e.grad.clone()
    for v in list(p.values()) + [e]:
        v.grad = None
    pr = ref.head_forward(p, e, E, N, K, Q, R, head, bf16=True)
    lr = ref.loss_fn(loss_type)(pr, labels.long())
    (lr * 3.0).backward()
    assert abs(float(loss) - float(lr)) <= 2e-2 * abs(float(lr)) + 1e-6
    thr = 0.5 if loss_type == "ce_nota" else None   # ce_nota: NOTA predicted below the score 0.5
    assert abs(float(acc) - float(ref.accuracy(probs, labels.long(), thr))) < 1e-6
    assert _nrel(ge, e.grad) < 2e-2
    for k in p:   # paper head + CE: the shared bias cancels in the softmax (its exact gradient is 0)
        assert _nrel(got[k], p[k].grad) < 2e-2 or float((got[k] - p[k].grad).abs().max()) < 1e-5, k
