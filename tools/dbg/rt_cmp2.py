"""Routing forward on the head test's exact inputs: per-item max-abs error vs fp64 oracle (debug aid)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from test_kernels_gpu import _problem, DEV
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.models import reference as ref
for (N, K, Q) in [(10, 5, 2), (5, 2, 5)]:
    B = 4
    cfg, data, model, dd, inst, labels = _problem(B=B, N=N, K=K, Q=Q, head="reference")
    H = 2 * cfg.hidden_size
    S = inst.shape[0]
    torch.manual_seed(0)
    e = (torch.randn(S, H, device=DEV) * 0.5)
    Ws = model.pdict()["W_s"].detach().contiguous()
    cls = ops().routing_fwd(e, Ws, B, N, K, Q, 3, 0)
    ev = e.double().view(B, N * K + N * Q, H)
    cr = ref.dynamic_routing(ev[:, : N * K].reshape(B, N, K, H), Ws.double(), 3)
    err = (cls.double() - cr).abs().amax(-1) / cr.abs().amax()
    print(N, K, Q, "H", H, "Ws absmax", float(Ws.abs().max()), "per-item max err:", [f"{x:.1e}" for x in err.flatten().tolist()])
