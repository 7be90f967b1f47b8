"""Compare routing kernels of the current library against the oracle for one shape (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.models import reference as ref
dev = "cuda"
for (N, K, Q, H, B) in [(10, 5, 2, 40, 4), (5, 5, 5, 40, 4), (5, 3, 2, 40, 6)]:
    torch.manual_seed(0)
    S = B * (N * K + N * Q)
    e = torch.randn(S, H, device=dev) * 0.5
    Ws = torch.randn(H, H, device=dev) * 0.2
    cls = ops().routing_fwd(e, Ws, B, N, K, Q, 3, 0)
    ev = e.view(B, N * K + N * Q, H)
    er = e.clone().requires_grad_(True)
    Wr = Ws.clone().requires_grad_(True)
    cr = ref.dynamic_routing(er.view(B, N * K + N * Q, H)[:, : N * K].reshape(B, N, K, H), Wr, 3)
    dc = torch.randn_like(cr)
    (cr * dc).sum().backward()
    de = torch.zeros_like(e)
    slab = ops().routing_bwd(e, Ws, dc.contiguous(), de, B, N, K, Q, 3, 0)
    rel = lambda a, b: float((a - b).norm() / b.norm())
    sup = torch.cat([torch.arange(b * (N * K + N * Q), b * (N * K + N * Q) + N * K) for b in range(B)]).to(dev)
    print(N, K, H, "cls", rel(cls, cr.detach()), "de", rel(de[sup], er.grad[sup]), "dWs", rel(slab.sum(0), Wr.grad),
          "de_query_zero", float(de.abs().sum() - de[sup].abs().sum()))
