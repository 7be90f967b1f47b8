"""Debug: every head gradient's error vs the oracle (the assertion order of test_head_forward_backward hides
all but the first).  usage (GPU): python tools/dbg/head_grads.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import torch  # noqa: E402
import test_kernels_gpu as T  # noqa: E402
from induction_network_on_fewrel_amd.models import reference as ref  # noqa: E402
from induction_network_on_fewrel_amd.ops import ops  # noqa: E402
from induction_network_on_fewrel_amd.ops.head import head as head_fn  # noqa: E402

QUICK = os.environ.get("INA_DBG_QUICK") == "1"
for head in ("reference",) if QUICK else ("reference", "paper"):
    for shape in [(5, 2, 5)] if QUICK else [(5, 2, 5), (10, 5, 2), (5, 5, 5, 9, 600)]:
        N, K, Q = shape[:3]
        B = shape[4] if len(shape) > 4 else 4
        cfg, data, model, dd, inst, labels = T._problem(B=B, N=N, K=K, Q=Q, head=head,
                                                        slices=shape[3] if len(shape) > 3 else 100)
        H = 2 * cfg.hidden_size
        S = inst.shape[0]
        torch.manual_seed(0)
        e = (torch.randn(S, H, device="cuda") * 0.5).requires_grad_(True)
        p = model.pdict()
        probs = head_fn(e, p, dict(E=B, N=N, K=K, Q=Q, iters=3, paper=(head == "paper")))
        dp = torch.randn_like(probs)
        (probs * dp).sum().backward()
        pr = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
        er = e.detach().clone().requires_grad_(True)
        ev = er.view(B, N * K + N * Q, H)
        cls = ref.dynamic_routing(ev[:, : N * K].reshape(B, N, K, H), pr["W_s"], 3)
        cls_k = ops().routing_fwd(e.detach().contiguous(), p["W_s"].detach().contiguous(), B, N, K, Q, 3, 0)
        cls = cls + (cls_k.view_as(cls) - cls).detach()
        probs_r = ref.relation_probs(cls, ev[:, N * K:], pr["M"], pr["ntn_w"], pr["ntn_b"], head, bf16=True)
        (probs_r * dp).sum().backward()
        qrows = torch.cat([torch.arange(b * (N * K + N * Q) + N * K, (b + 1) * (N * K + N * Q)) for b in range(B)])
        srows = torch.cat([torch.arange(b * (N * K + N * Q), b * (N * K + N * Q) + N * K) for b in range(B)])
        res = {"probs": T._relerr(probs.detach(), probs_r.detach()),
               "e_query": T._relerr(e.grad[qrows], er.grad[qrows]), "e_support": T._relerr(e.grad[srows], er.grad[srows])}
        for k, a, b in (("W_s", p["W_s"].grad, pr["W_s"].grad), ("M", p["M"].grad, pr["M"].grad),
                        ("w", p["ntn_w"].grad, pr["ntn_w"].grad), ("b", p["ntn_b"].grad, pr["ntn_b"].grad)):
            res[k] = T._relerr(a, b)
        print(head, shape, {k: f"{v:.2e}" for k, v in res.items()}, flush=True)
