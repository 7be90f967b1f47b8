"""CPU check of the wide head's orchestration (ops/wide.py::_wide_head_forward / _backward): the four
head_wide.hip kernels are replaced by float32 PyTorch emulations of their documented semantics and the
bf16 GEMM operands by fp32, so the layouts (M' = M permuted to [a, s*H + b'], T columns c*h + s, the
reference FC's row s*N + c, the dM un-permute, the support / query split of de) are pinned exactly
against models/reference.py::head_forward's autograd."""
import pytest
import torch

import induction_network_on_fewrel_amd.ops.wide as W
from induction_network_on_fewrel_amd.models import reference as ref


class _EmuOps:
    def routing_wide_ok(self, K, H, R):
        return True

    def transpose12(self, x, bf16):
        return x.permute(0, 2, 1).contiguous()   # (the emulation keeps fp32 where the kernel writes bf16)

    def ntn_wide_epi_ok(self, N, paper):
        return True

    def routing_wide_fwd(self, eh, items, K, R):
        H = eh.shape[1]
        c = ref.dynamic_routing(eh.view(items, 1, K, H), torch.eye(H), R).view(items, H)
        return c, c.clone()

    def routing_wide_bwd(self, eh, dcls, items, K, R):
        H = eh.shape[1]
        with torch.enable_grad():
            x = eh.detach().view(items, K, H).clone().requires_grad_(True)
            c = ref.dynamic_routing(x.view(items, 1, K, H), torch.eye(H), R).view(items, H)
            (g,) = torch.autograd.grad(c, x, dcls)
        return g.reshape(items * K, H)

    def ntn_wide_epi_fwd(self, T, N, h, w, b, paper):
        rows = T.numel() // (N * h)
        V = torch.relu(T.view(rows, N, h))
        if paper:
            z = (V * w.view(1, 1, h)).sum(2) + b
        else:
            z = V.permute(0, 2, 1).reshape(rows, h * N) @ w.view(h * N, N) + b
        return torch.sigmoid(z)

    def ntn_wide_epi_bwd(self, T, N, h, w, dz, g, paper):
        rows = T.numel() // (N * h)
        Tv = T.view(rows, N, h)
        dzs = dz * (float(g) if g.numel() else 1.0)
        if paper:
            gv = w.view(1, 1, h) * dzs.view(rows, N, 1)
        else:
            gv = (w.view(h, N, N)[None] * dzs.view(rows, 1, 1, N)).sum(3).permute(0, 2, 1)
        dT = torch.where(Tv > 0, gv, torch.zeros_like(gv)).reshape(rows, N * h)
        T.clamp_(min=0)
        return dT, dzs


class _Fp32Torch:
    """torch with bf16 -> fp32 and the out_dtype GEMM overloads (CUDA-only in torch) on the CPU."""
    bfloat16 = torch.float32

    def __getattr__(self, k):
        return getattr(torch, k)

    @staticmethod
    def mm(a, b, out_dtype=None):
        return torch.mm(a, b)

    @staticmethod
    def bmm(a, b, out_dtype=None):
        return torch.bmm(a, b)


@pytest.fixture
def emulated(monkeypatch):
    monkeypatch.setattr(W, "ops", lambda: _EmuOps())
    monkeypatch.setattr(W, "torch", _Fp32Torch())


@pytest.mark.parametrize("head", ["reference", "paper"])
@pytest.mark.parametrize("N,K,Q", [(5, 5, 20), (3, 1, 2)])
def test_wide_head_layouts_exact(emulated, head, N, K, Q):
    E, H, h, R = 3, 32, 12, 3
    g = torch.Generator().manual_seed(N * 10 + K)
    p = dict(W_s=torch.randn(H, H, generator=g) / H ** 0.5, M=torch.randn(H, H, h, generator=g) * 0.2,
             ntn_w=torch.randn(h * N, N, generator=g) * 0.3 if head == "reference" else torch.randn(h, 1, generator=g),
             ntn_b=torch.randn(N if head == "reference" else 1, generator=g) * 0.1)
    p = {k: v.requires_grad_(True) for k, v in p.items()}
    e = (torch.randn(E * (N * K + N * Q), H, generator=g) * 0.5).requires_grad_(True)
    probs = W.HeadWideProbsFn.apply(e, p["W_s"], p["M"], p["ntn_w"], p["ntn_b"], (E, N, K, Q, R, head == "paper"))
    gout = torch.randn(probs.shape, generator=g)
    (probs * gout).sum().backward()
    got = {k: v.grad.clone() for k, v in p.items()}
    ge = e.grad.clone()
    for v in list(p.values()) + [e]:
        v.grad = None
    pr = ref.head_forward(p, e, E, N, K, Q, R, head)
    (pr * gout).sum().backward()
    assert torch.allclose(probs, pr, atol=1e-6)
    assert torch.allclose(ge, e.grad, rtol=1e-4, atol=1e-6)
    for k in p:
        assert torch.allclose(got[k], p[k].grad, rtol=1e-4, atol=1e-6), k


@pytest.mark.parametrize("loss_type", ["mse", "ce"])
def test_wide_head_loss_backward_scale(emulated, monkeypatch, loss_type):
    """HeadWideLossFn's backward scales dz by the upstream gradient (ina.head_loss emulated)."""
    E, N, K, Q, H, h, R = 2, 4, 2, 3, 16, 8, 3

    def head_loss(probs, labels, scale, dz, out, part, blocks, ce):
        with torch.enable_grad():
            pr = probs.detach().clone().requires_grad_(True)
            z = torch.log(pr) - torch.log1p(-pr)
            zz = z.detach().requires_grad_(True)
            p2 = torch.sigmoid(zz)
            lf = ref.ce_loss if ce else ref.mse_loss
            loss = lf(p2.view(E, N * Q, N), labels.view(E, N * Q).long())
            (gz,) = torch.autograd.grad(loss, zz)
        dz.copy_(gz)
        out[0] = loss.detach()
        out[1] = ref.accuracy(probs, labels.long())

    emu = _EmuOps()
    emu.head_loss = head_loss
    monkeypatch.setattr(W, "ops", lambda: emu)
    g = torch.Generator().manual_seed(3)
    p = {k: v.requires_grad_(True) for k, v in dict(
        W_s=torch.randn(H, H, generator=g) / H ** 0.5, M=torch.randn(H, H, h, generator=g) * 0.3,
        ntn_w=torch.randn(h * N, N, generator=g) * 0.3, ntn_b=torch.randn(N, generator=g) * 0.1).items()}
    e = (torch.randn(E * (N * K + N * Q), H, generator=g) * 0.5).requires_grad_(True)
    labels = torch.randint(0, N, (E, N * Q), generator=g).int()
    loss, acc, _ = W.HeadWideLossFn.apply(e, p["W_s"], p["M"], p["ntn_w"], p["ntn_b"], labels,
                                          (E, N, K, Q, R, False), loss_type, "mean")
    (2.5 * loss).backward()
    got = {k: v.grad.clone() for k, v in p.items()}
    for v in p.values():
        v.grad = None
    lf = ref.ce_loss if loss_type == "ce" else ref.mse_loss
    lr = lf(ref.head_forward(p, e, E, N, K, Q, R, "reference"), labels.long())
    (2.5 * lr).backward()
    assert abs(float(loss) - float(lr)) < 1e-5
    for k in p:
        assert torch.allclose(got[k], p[k].grad, rtol=1e-3, atol=1e-6), k
