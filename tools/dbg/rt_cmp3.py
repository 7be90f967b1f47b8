"""Head test sequence with a routing check before each head call (debug aid)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_kernels_gpu import _problem, DEV, _relerr
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.ops.head import head as head_fn
from induction_network_on_fewrel_amd.models import reference as ref
for (N, K, Q) in [(5, 2, 5), (5, 1, 5), (10, 5, 2)]:
  for hd in ["reference", "paper"]:
    B = 4
    cfg, data, model, dd, inst, labels = _problem(B=B, N=N, K=K, Q=Q, head=hd)
    H = 2 * cfg.hidden_size
    S = inst.shape[0]
    torch.manual_seed(0)
    e = (torch.randn(S, H, device=DEV) * 0.5).requires_grad_(True)
    p = model.pdict()
    Ws = p["W_s"].detach().contiguous()
    cls = ops().routing_fwd(e.detach(), Ws, B, N, K, Q, 3, 0)
    ev = e.detach().view(B, N * K + N * Q, H)
    cr = ref.dynamic_routing(ev[:, : N * K].reshape(B, N, K, H), Ws, 3)
    probs = head_fn(e, p, dict(E=B, N=N, K=K, Q=Q, iters=3, paper=(hd == "paper")))
    probs_r = ref.relation_probs(cr, ev[:, N * K:], p["M"].detach(), p["ntn_w"].detach(), p["ntn_b"].detach(), hd, bf16=True)
    cls2 = ops().routing_fwd(e.detach(), Ws, B, N, K, Q, 3, 0)
    torch.cuda.synchronize()
    print(N, K, Q, hd, "cls err", _relerr(cls, cr), "cls2 err", _relerr(cls2, cr), "probs err", _relerr(probs.detach(), probs_r))
