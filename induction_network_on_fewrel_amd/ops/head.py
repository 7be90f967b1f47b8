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
        dcls, dp, dw_slab = o.ntn_bwd(cls, e, mpack, m2pack, wtpack, wvec, dz, de, E, N, K, Q, h, paper, 0, None, None)
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


class HeadLossFn(torch.autograd.Function):
    """Routing + NTN + sigmoid + MSE loss + accuracy in one autograd node (StepGlue training path).

    forward:  routing_fwd -> ntn_fwd -> ina.head_loss (loss, accuracy, dz = dL/dlogit and its row
              sum = the NTN bias gradient, all in one launch; reference model/graph.py:88-95)
    backward: ntn_bwd scales dz by the upstream loss gradient on the device and also emits the bf16
              copy of the class vectors for the dM GEMM (fp32 output); every parameter gradient is
              queued on the StepGlue for the step's single slab_scatter_add.
    Returns (loss, accuracy, probs); accuracy and probs are not differentiable."""

    @staticmethod
    def forward(ctx, e, Ws, M, w, b, labels, meta):
        o = ops()
        E, N, K, Q, R = meta["E"], meta["N"], meta["K"], meta["Q"], meta["iters"]
        paper = bool(meta["paper"])
        glue, pk = meta["glue"], meta["packs"]
        H, _, h = M.shape
        e = e.contiguous()
        Wsd = Ws.detach().contiguous()
        cls = o.routing_fwd(e, Wsd, E, N, K, Q, R, 0)
        mpack, m2pack = pk["mpack"], pk["m2pack"]
        if paper:
            wpack = wtpack = torch.empty(0, dtype=torch.bfloat16, device=e.device)
            wvec = w.detach().reshape(-1).float().contiguous()
        else:
            wpack, wtpack = pk["wpack"], pk["wtpack"]
            wvec = torch.empty(0, dtype=torch.float32, device=e.device)
        probs = o.ntn_fwd(cls, e, mpack, wpack, wvec, b.detach().float().contiguous(), E, N, K, Q, h, paper, 0)
        rows = E * N * Q
        ce = meta.get("loss_type", "mse") == "ce"
        if meta.get("reduction", "mean") == "mean":
            scale = 1.0 / rows if ce else 1.0 / (rows * N)
        else:
            scale = 1.0 / max(1, E)
        dz = torch.empty_like(probs)
        out = torch.empty(N + 3, dtype=torch.float32, device=e.device)
        o.head_loss(probs, labels.reshape(-1), scale, dz, out, glue.loss_part, _loss_blocks(glue, rows), ce)
        ctx.save_for_backward(e, Wsd, cls, mpack, m2pack, wtpack, wvec, dz, out)
        ctx.meta = dict(meta, H=H, h=h)
        ctx.set_materialize_grads(False)   # no zero-fill launches for the non-differentiable outputs
        loss, acc = out[0], out[1]
        ctx.mark_non_differentiable(acc, probs)
        return loss, acc, probs

    @staticmethod
    def backward(ctx, gloss, _gacc, _gprobs):
        o = ops()
        e, Ws, cls, mpack, m2pack, wtpack, wvec, dz, out = ctx.saved_tensors
        m = ctx.meta
        E, N, K, Q, R, H, h = m["E"], m["N"], m["K"], m["Q"], m["iters"], m["H"], m["h"]
        paper = bool(m["paper"])
        glue, p = m["glue"], m["pdict"]
        g = gloss.reshape(1).float().contiguous()
        de = torch.empty_like(e)
        cls_bf = torch.empty(E * N, H, dtype=torch.bfloat16, device=e.device)
        dcls, dp, dw_slab = o.ntn_bwd(cls, e, mpack, m2pack, wtpack, wvec, dz, de, E, N, K, Q, h, paper, 0, g, cls_bf)
        # dM = C^T dP over K = E*N rows: split-K as a batched GEMM [ns, H, h*H] (a plain [H=40] x
        # [h*H=4000] GEMM has only ~63 output tiles -- a quarter of the CUs streaming the 82 MB dP); the
        # ns partial slabs are summed by the glue's deterministic slab scatter-add
        ns = _dm_splits(E * N)
        dMf = torch.bmm(cls_bf.view(ns, -1, H).transpose(1, 2), dp.view(ns, -1, dp.shape[1]),
                        out_dtype=torch.float32)                          # [ns, H, h*H] (col s*H + b)
        slab = o.routing_bwd(e, Ws, dcls, de, E, N, K, Q, R, 0)
        glue.add(dw_slab, glue.map_identity(p["ntn_w"]), dw_slab.shape[0])
        glue.add(out[2 + N:3 + N] if paper else out[2:2 + N], glue.map_identity(p["ntn_b"]), 1, scale=g)
        glue.add(slab, glue.map_identity(p["W_s"]), slab.shape[0])
        glue.add(dMf, glue.map_ntn_M(p["M"]), ns)
        ov = m.get("overlap")
        if ov is not None:   # DP: scatter the head's gradients now and start their all-reduce (bucket 0)
            glue.flush()
            ov.ready(0)
        return de, None, None, None, None, None, None


def _dm_splits(rows: int) -> int:
    """Split-K factor of the dM GEMM: >= 1024 (episode, class) rows per split, dividing ``rows``."""
    for ns in (8, 4, 2):
        if rows % ns == 0 and rows // ns >= 1024:
            return ns
    return 1


def _loss_blocks(glue, rows: int) -> int:
    return max(1, min(glue.LOSS_BLOCKS, (rows + 255) // 256))


def head_loss(e, params, labels, meta):
    return HeadLossFn.apply(e, params["W_s"], params["M"], params["ntn_w"], params["ntn_b"], labels, meta)
