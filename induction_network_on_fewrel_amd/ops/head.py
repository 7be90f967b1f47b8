"""Induction + relation head on the GPU path: dynamic routing -> neural tensor layer -> sigmoid.

forward:  routing_fwd -> ntn_fwd (slice tiles x stacked episodes, bf16 MFMA; csrc/kernels/ntn.hip)
backward: ntn_bwd (dC, dQ, dw slab, dP) -> dM = C^T dP (reduction GEMM over the E*N class rows)
          -> routing_bwd (exact reverse through all routing iterations, dW_s slab)
The gradient wrt the sentence embeddings is written by ntn_bwd (query rows) and routing_bwd
(support rows) into ONE buffer -- no zero-fill and no add of two sparse gradients.

Reference: model/layer_module.py:8-47 (NTN), :101-162 (routing); model/graph.py:57-86.
"""
from __future__ import annotations

import torch

from ._ext import ops
from .encoder import _route_grad
from .packing import _ntn_dw_idx, _on, pack_ntn_tiles


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
        tiles = pack_ntn_tiles(M, w, N, paper)
        probs = o.ntn_fwd(cls, e, tiles, b.detach().float().contiguous(), E, N, K, Q, h, paper, 0)
        ctx.save_for_backward(e, Wsd, cls, tiles, probs)
        ctx.meta = dict(meta, H=H, h=h)
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        o = ops()
        e, Ws, cls, tiles, probs = ctx.saved_tensors
        m = ctx.meta
        E, N, K, Q, R, H, h = m["E"], m["N"], m["K"], m["Q"], m["iters"], m["H"], m["h"]
        paper = bool(m["paper"])
        dz = (dprobs * probs * (1.0 - probs)).float().contiguous()
        de = torch.empty_like(e)
        dcls, dp, dw_slab, cls_bf = o.ntn_bwd(cls, e, tiles, dz, de, E, N, K, Q, h, paper, 0, None)
        # dM[a][b][s] = sum_{(e,c)} C[(e,c)][a] dP[(e,c)][s*H + b]   (gemm_tn.hip, split slabs)
        dMf = o.gemm_tn_slab(cls_bf, dp, H, 0).sum(0)   # [H, h*H]
        dM = dMf.view(H, h, H).permute(0, 2, 1).contiguous()
        di = _on(_ntn_dw_idx(h, N, paper), e.device)
        ok = di >= 0
        dw = torch.zeros(h if paper else h * N * N, dtype=torch.float32, device=e.device)
        dw.index_add_(0, di[ok], dw_slab.sum(0)[ok])
        if paper:
            dw = dw.view(h, 1)
            db = dz.sum().view(1)
        else:
            dw = dw.view(h * N, N)
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
              class vectors and dP for the dM reduction GEMM (gemm_tn.hip, fp32 split slabs); every
              parameter gradient is queued on the StepGlue for the step's single slab_scatter_add.
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
        tiles = pk["ntn_tiles"]
        probs = o.ntn_fwd(cls, e, tiles, b.detach().float().contiguous(), E, N, K, Q, h, paper, 0)
        rows = E * N * Q
        lt = meta.get("loss_type", "mse")
        ce = lt != "mse"   # scale: mean over the queries (ce, ce_nota) or over queries x classes (mse)
        mode = {"mse": 0, "ce": 1, "ce_nota": 2}[lt]
        if meta.get("reduction", "mean") == "mean":
            scale = 1.0 / rows if ce else 1.0 / (rows * N)
        else:
            scale = 1.0 / max(1, E)
        dz = torch.empty_like(probs)
        out = torch.empty(N + 3, dtype=torch.float32, device=e.device)
        o.head_loss(probs, labels.reshape(-1), scale, dz, out, glue.loss_part, _loss_blocks(glue, rows), mode)
        ctx.save_for_backward(e, Wsd, cls, tiles, dz, out)
        ctx.meta = dict(meta, H=H, h=h)
        ctx.set_materialize_grads(False)   # no zero-fill launches for the non-differentiable outputs
        loss, acc = out[0], out[1]
        ctx.mark_non_differentiable(acc, probs)
        return loss, acc, probs

    @staticmethod
    def backward(ctx, gloss, _gacc, _gprobs):
        o = ops()
        e, Ws, cls, tiles, dz, out = ctx.saved_tensors
        m = ctx.meta
        E, N, K, Q, R, H, h = m["E"], m["N"], m["K"], m["Q"], m["iters"], m["H"], m["h"]
        paper = bool(m["paper"])
        glue, p = m["glue"], m["pdict"]
        g = gloss.reshape(1).float().contiguous()
        de = torch.empty_like(e)
        dcls, dp, dw_slab, cls_bf = o.ntn_bwd(cls, e, tiles, dz, de, E, N, K, Q, h, paper, 0, g)
        # dM = C^T dP over the E*N class rows: the split-K reduction GEMM of gemm_tn.hip -> slabs [ns, H, h*H]
        # (col s*H + b), summed by the glue's deterministic slab scatter-add
        dMf = o.gemm_tn_slab(cls_bf, dp, H, 0)
        ns = dMf.shape[0]
        slab = o.routing_bwd(e, Ws, dcls, de, E, N, K, Q, R, 0)
        glue.add(dw_slab, glue.map_ntn_dw(p["ntn_w"], h, N, paper), dw_slab.shape[0])
        glue.add(out[2 + N:3 + N] if paper else out[2:2 + N], glue.map_identity(p["ntn_b"]), 1, scale=g)
        glue.add(slab, glue.map_identity(p["W_s"]), slab.shape[0])
        glue.add(dMf, glue.map_ntn_M(p["M"]), ns)
        ov = m.get("overlap")
        if ov is not None:   # DP: scatter the head's gradients now and start their all-reduce (bucket 0)
            glue.flush()
            ov.ready(0)
        return de, None, None, None, None, None, None


def _loss_blocks(glue, rows: int) -> int:
    return max(1, min(glue.LOSS_BLOCKS, (rows + 255) // 256))


def head_loss(e, params, labels, meta):
    return HeadLossFn.apply(e, params["W_s"], params["M"], params["ntn_w"], params["ntn_b"], labels, meta)
