"""Induction + relation head on the GPU path: dynamic routing -> neural tensor layer -> sigmoid.

forward:  routing_fwd (one wave / episode) -> ntn_fwd (one wave / episode, chained bf16 MFMAs)
backward: ntn_bwd (dC, dQ, per-episode dw, dP) -> dM = C^T dP (library GEMM over E*N)
          -> routing_bwd (exact reverse through all routing iterations, dW_s slab)
The gradient wrt the sentence embeddings is written by ntn_bwd (query rows) and routing_bwd
(support rows) into ONE buffer -- no zero-fill and no add of two sparse gradients.

Reference: model/layer_module.py:8-47 (NTN), :101-162 (routing); model/graph.py:57-86.
"""
from __future__ import annotations

import torch

from ._ext import ops
from .encoder import _route_grad
from .packing import pack_ntn_M, pack_ntn_w


class HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, e, Ws, M, w, b, meta):
        """meta = dict(E, N, K, Q, iters, paper)."""
        o = ops()
        E, N, K, Q, R = meta["E"], meta["N"], meta["K"], meta["Q"], meta["iters"]
        paper = bool(meta["paper"])
        H, _, h = M.shape
        e = e.contiguous()
        Wsd = Ws.detach().contiguous()
        cls = o.routing_fwd(e, Wsd, E, N, K, Q, R, 0)
        mpack, m2pack = pack_ntn_M(M)
        if paper:
            wpack = wtpack = torch.empty(0, dtype=torch.bfloat16, device=e.device)
            wvec = w.detach().reshape(-1).float().contiguous()
        else:
            wpack, wtpack = pack_ntn_w(w, h, N)
            wvec = torch.empty(0, dtype=torch.float32, device=e.device)
        probs = o.ntn_fwd(cls, e, mpack, wpack, wvec, b.detach().float().contiguous(), E, N, K, Q, h, paper, 0)
        ctx.save_for_backward(e, Wsd, cls, mpack, m2pack, wtpack, wvec, probs)
        ctx.meta = dict(meta, H=H, h=h)
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        o = ops()
        e, Ws, cls, mpack, m2pack, wtpack, wvec, probs = ctx.saved_tensors
        m = ctx.meta
        E, N, K, Q, R, H, h = m["E"], m["N"], m["K"], m["Q"], m["iters"], m["H"], m["h"]
        paper = bool(m["paper"])
        dz = (dprobs * probs * (1.0 - probs)).float().contiguous()
        de = torch.empty_like(e)
        dcls, dp, dw_slab = o.ntn_bwd(cls, e, mpack, m2pack, wtpack, wvec, dz, de, E, N, K, Q, h, paper, 0)
        # dM[a][b][s] = sum_{(e,c)} C[(e,c)][a] dP[(e,c)][s*H + b]
        dMf = torch.matmul(cls.reshape(E * N, H).t().to(torch.bfloat16), dp).float()   # [H, h*H]
        dM = dMf.view(H, h, H).permute(0, 2, 1).contiguous()
        if paper:
            dw = dw_slab.sum(0).view(h, 1)
            db = dz.sum().view(1)
        else:
            dw = dw_slab.sum(0).reshape(h * N, N)
            db = dz.sum((0, 1))
        slab = o.routing_bwd(e, Ws, dcls, de, E, N, K, Q, R, 0)
        dWs = slab.sum(0)
        return (de, _route_grad(m, "W_s", dWs), _route_grad(m, "M", dM), _route_grad(m, "ntn_w", dw),
                _route_grad(m, "ntn_b", db), None)


def head(e, params, meta):
    return HeadFn.apply(e, params["W_s"], params["M"], params["ntn_w"], params["ntn_b"], meta)
