"""BERT encoder on the GPU path: hand-written gfx950 kernels + hipBLASLt GEMMs (bf16).

GEMMs (csrc/kernels/gemm.hip is one NT / NN / TN kernel family): every weight gradient dW = dy^T x runs on the
own TN split-K kernel (fp32 slabs summed into the flat gradient: 377-500 vs 469-581 us for hipBLASLt at the four
BERT-base shapes, BERT 111.7 vs 109.6 episodes/s, profiles/r6_gemm, r6_bert); the FFN-up forward (bias + GELU)
and its dgrad (GELU' + db) on the own NT kernel; the other forwards / dgrads on hipBLASLt by default
(INA_BERT_OWN_NT=1 / INA_BERT_OWN_NN=1 put them on the own kernels: 1-2% slower end to end, see _own_nn_ok).

Per layer (post-LN BERT, models/bert.py is the oracle):
    qkv = x Wqkv^T + bqkv            torch.addmm (bf16 -> hipBLASLt); Wqkv is ONE [3Hd, Hd] view of the
                                     flat bf16 weight copy (q/k/v are adjacent in the flat buffer)
    ctx = MHA(qkv)                   ina.bert_mha_fwd / _bwd   (fused, sequence in LDS, MFMA)
    x1  = LN(x + drop(ctx Wo^T+bo))  addmm + ina.bert_ln_res_fwd / _bwd
    h   = gelu(x1 W1^T + b1)         _Ffn (default; INA_BERT_OWN_GEMM=0: mm + ina.bert_bias_gelu_fwd / _bwd): the
                                     own gemm.hip kernel with bias + GELU / GELU' + db in its epilogues
    x2  = LN(x1 + drop(h W2^T+b2))   addmm + ina.bert_ln_res_fwd / _bwd
Embeddings: ina.bert_embed_ln_fwd / _bwd (gather by instance index, no host copies); the word-table
gradient is scattered with index_add_ straight into the flat gradient buffer.

Weights: the encoder layers' fp32 masters are cast to bf16 ONCE per step as one contiguous region of
the flat parameter buffer (outside autograd).  ``_Linear`` computes dW / db with fp32-output GEMMs and
adds them straight into the flat gradient buffer (no bf16 weight-gradient tensors, no autograd slice
accumulation).  LayerNorm / GELU-bias / embedding tables stay fp32.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from ._ext import ops
from .encoder import _route_grad


def _glue_maps(meta, names):
    """The StepGlue and the flat-gradient maps of ``names`` when every one of them is routed to the flat
    gradient buffer (trainer path), else (None, None): the caller reduces with torch and routes."""
    glue, views = meta.get("glue"), meta.get("grad_views")
    if glue is None or views is None or any(n is None or n not in views for n in names):
        return None, None
    return glue, [glue.map_grad(views[n]) for n in names]


def _contiguous_region(ts: List[torch.Tensor]) -> Optional[torch.Tensor]:
    """A 1-D view spanning ts if they are back-to-back in one storage (flat buffer), else None."""
    base = ts[0]
    off = base.storage_offset()
    total = 0
    for t in ts:
        if (t.untyped_storage().data_ptr() != base.untyped_storage().data_ptr() or t.storage_offset() != off + total
                or not t.is_contiguous()):
            return None
        total += t.numel()
    return torch.as_strided(base.detach(), (total,), (1,), off)


def _own_wgrad_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """Shapes the own TN split-K GEMM takes (csrc/kernels/gemm.hip: 16-byte column chunks, bf16 GPU rows);
    INA_BERT_OWN_WGRAD=0 selects hipBLASLt (A/B)."""
    return (os.environ.get("INA_BERT_OWN_WGRAD", "1") != "0" and dy.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.shape[1] % 8 == 0
            and x.shape[1] % 8 == 0 and dy.stride(1) == 1 and x.stride(1) == 1 and dy.stride(0) % 8 == 0
            and x.stride(0) % 8 == 0 and dy.shape[0] > 0)


def _wgrad_parts(dy: torch.Tensor, x: torch.Tensor):
    """fp32 split-K partials [splits, o, i] of dy^T x (own TN GEMM: one round of 256x256 output tiles over the
    CUs, K = tokens split so every CU has a tile), or None where _wgrad uses one GEMM."""
    if _own_wgrad_ok(dy, x):
        return ops().gemm_wgrad(dy, x, 0)
    T, o = dy.shape
    i = x.shape[1]
    nc = 16
    if T % nc != 0 or T < 4096:
        return None
    return torch.bmm(dy.view(nc, T // nc, o).transpose(1, 2), x.view(nc, T // nc, i), out_dtype=torch.float32)


def _wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW = dy^T x in fp32.  K = tokens is the long dimension and the output has few 256x256 tiles, so the
    reduction is split-K (own TN GEMM slabs: 380 vs 467 us for hipBLASLt's 16-chunk bmm at the QKV shape,
    profiles/r6_gemm) + an ordered sum."""
    part = _wgrad_parts(dy, x)
    if part is None:
        return torch.mm(dy.t(), x, out_dtype=torch.float32)
    return part.sum(0)


def _own_nn_ok(dy: torch.Tensor, W: torch.Tensor) -> bool:
    """The own NN dgrad GEMM, opt-in (INA_BERT_OWN_NN=1).  Measured in the BERT step (profiles/r6_bert1): 2% slower
    than hipBLASLt -- ~6% tile quantization at N = 768 (400 x 3 tiles over 256 CUs: 5 rounds for 4.69 of work;
    hipBLASLt's stream-K kernels split the last round), and its GELU' epilogue at N = 3072 takes 875 us against
    761 us for the NT kernel's (+ a 5 us transposed weight copy)."""
    return (os.environ.get("INA_BERT_OWN_NN", "0") == "1" and dy.is_cuda and dy.dtype == torch.bfloat16 and W.dtype == torch.bfloat16 and dy.is_contiguous()
            and W.is_contiguous() and dy.shape[1] % 64 == 0 and W.shape[1] % 8 == 0)


def _dgrad(dy: torch.Tensor, W: torch.Tensor, res: Optional[torch.Tensor]) -> torch.Tensor:
    """dx = dy W (+ res, in place): the own NN GEMM (W [out][in] read K-major, residual added in its epilogue)."""
    if _own_nn_ok(dy, W) and (res is None or (res.is_contiguous() and res.dtype == torch.bfloat16)):
        return ops().gemm_nn(dy, W, None, res, 4 if res is not None else 0)[0]
    return res.addmm_(dy, W) if res is not None else torch.mm(dy, W)


def _own_nt() -> bool:
    """Forward linears on the own NT GEMM (INA_BERT_OWN_NT=1) instead of hipBLASLt addmm."""
    return os.environ.get("INA_BERT_OWN_NT", "0") == "1"


def _fwd_linear(x: torch.Tensor, Wb: torch.Tensor, bias: Optional[torch.Tensor], bb: Optional[torch.Tensor]):
    """y = x W^T (+ b): own NT GEMM with the fp32 bias in its epilogue (INA_BERT_OWN_NT=1) or hipBLASLt."""
    if (_own_nt() and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.shape[1] % 64 == 0
            and Wb.shape[0] % 8 == 0):
        return ops().bert_gemm(x, Wb, bias, None, 0)[0]
    return torch.addmm(bb, x, Wb.t()) if bb is not None else torch.mm(x, Wb.t())


class _Linear(torch.autograd.Function):
    """y = x W^T (+ b) with bf16 operands taken from the per-step bf16 weight copy.

    W may be the row-concatenation of several fp32 parameters (fused QKV).  Backward computes dW and
    db in fp32 (hipBLASLt bf16 GEMM with fp32 output) and either adds them straight into the flat
    gradient buffer spans (trainer path) or returns them per parameter (plain autograd)."""

    @staticmethod
    def forward(ctx, x, Wb, bb, gW, gb, nw, on_done, db_ext, dx_acc, bf32, *params):
        """db_ext: the bias gradient is produced by the consumer's backward (_LnRes / _Mha: column sums
        of the same dy, fused into their kernels), so this backward skips the dy.sum(0) pass.
        dx_acc: a _ResGrad holder; x's other gradient (the residual branch of the LayerNorm that also
        reads x) is added by the dgrad GEMM itself (addmm, beta = 1) instead of autograd's bf16 add."""
        y = _fwd_linear(x, Wb, bf32, bb)
        ctx.save_for_backward(x, Wb)
        ctx.cfg = (gW, gb, nw, [tuple(p.shape) for p in params], bb is not None and not db_ext, on_done, dx_acc)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, Wb = ctx.saved_tensors
        gW, gb, nw, shapes, has_b, on_done, dx_acc = ctx.cfg
        dy = dy.contiguous()
        res = dx_acc.take() if dx_acc is not None else None
        # in place into the LayerNorm's fresh residual gradient (the own NN GEMM's residual epilogue)
        dx = _dgrad(dy, Wb, res)
        db = dy.sum(0, dtype=torch.float32) if has_b else None
        outs = [None] * len(shapes)
        part = _wgrad_parts(dy, x) if gW is not None and gW.is_contiguous() else None
        if part is not None:
            # the split-K partials summed straight into the flat gradient span (one pass instead of
            # a reduction to a temporary plus an add)
            ops().slab_reduce(part, gW, True)
        elif gW is not None:
            gW.add_(_wgrad(dy, x).view(gW.shape))
        else:
            dW = _wgrad(dy, x)
            o = 0
            for i in range(nw):
                outs[i] = dW[o:o + shapes[i][0]]
                o += shapes[i][0]
        if has_b:
            if gb is not None:
                gb.add_(db)
            else:
                o = 0
                for i in range(nw, len(shapes)):
                    outs[i] = db[o:o + shapes[i][0]]
                    o += shapes[i][0]
        if on_done is not None:   # last backward op of a layer: its gradient bucket is final
            on_done()
        return (dx, None, None, None, None, None, None, None, None, None) + tuple(outs)


def _add_wgrad(gW, dy, x, shape):
    """dW = dy^T x (fp32) added into the flat gradient span gW, or returned (plain autograd)."""
    part = _wgrad_parts(dy, x) if gW is not None and gW.is_contiguous() else None
    if part is not None:
        ops().slab_reduce(part, gW, True)
        return None
    if gW is not None:
        gW.add_(_wgrad(dy, x).view(gW.shape))
        return None
    return _wgrad(dy, x).view(shape)


class _Ffn(torch.autograd.Function):
    """o = gelu(x W1^T + b1) W2^T + b2 on the own gfx950 GEMM (csrc/kernels/gemm.hip):

    forward : ONE kernel for x W1^T with bias + GELU + the bf16 pre-activation (aux) in its epilogue (replaces
              hipBLASLt mm + bert_bias_gelu_fwd), then h W2^T + b2 (hipBLASLt addmm).
    backward: ONE kernel for dh = do W2 with dpre = dh * GELU'(aux) and the b1 column-sum slab in its epilogue
              (replaces hipBLASLt mm + bert_bias_gelu_bwd); dx = dpre W1 (+ the residual gradient, as _Linear);
              dW1 / dW2 as _Linear's split-K fp32 GEMMs.
    b2's gradient comes from the following _LnRes (db_ext), as for the unfused path."""

    @staticmethod
    def forward(ctx, x, W1b, W2b, bb2, gW1, gW2, dx_acc, meta, b1name, b2f, W1, b1, W2):
        h, aux = ops().bert_gemm(x, W1b, b1.detach(), None, 1)
        o = _fwd_linear(h, W2b, b2f, bb2)
        ctx.save_for_backward(x, W1b, W2b, h, aux)
        ctx.cfg = (gW1, gW2, dx_acc, meta, b1name, tuple(W1.shape), tuple(W2.shape))
        return o

    @staticmethod
    def backward(ctx, do):
        x, W1b, W2b, h, aux = ctx.saved_tensors
        gW1, gW2, dx_acc, meta, b1name, s1, s2 = ctx.cfg
        do = do.contiguous()
        if _own_nn_ok(do, W2b):   # W2 [Hd][I] read K-major: no transposed copy
            dpre, slab = ops().gemm_nn(do, W2b, aux, None, 2)
        else:
            dpre, slab = ops().bert_gemm(do, W2b.t().contiguous(), None, aux, 2)
        dW2 = _add_wgrad(gW2, do, h, s2)
        res = dx_acc.take() if dx_acc is not None else None
        dx = _dgrad(dpre, W1b, res)
        dW1 = _add_wgrad(gW1, dpre, x, s1)
        glue, maps = _glue_maps(meta, [b1name])
        db1 = None
        if glue is not None:
            glue.add(slab, maps[0], slab.shape[0])
        else:
            db1 = _route_grad(meta, b1name, slab.sum(0))
        return dx, None, None, None, None, None, None, None, None, None, dW1, db1, dW2


def own_ffn_enabled(I: int, Hd: int) -> bool:
    """The own-GEMM FFN (default on since its 16-byte epilogue stores, round 5: BERT 10w5s 108.72 / 108.70 vs
    108.57 / 108.38 episodes/s with hipBLASLt + the separate bias / GELU passes, profiles/r5_widen/bert_ab;
    round 4 measured it at parity).  INA_BERT_OWN_GEMM=0 selects the hipBLASLt path.  Needs N = I a
    multiple of 256 and K = Hd a multiple of 64."""
    return os.environ.get("INA_BERT_OWN_GEMM", "1") != "0" and I % 256 == 0 and Hd % 64 == 0


class _ResGrad:
    """Hands a LayerNorm's residual-input gradient to the dgrad GEMM of the _Linear that reads the same
    x (both consumers of x; the LayerNorm's backward always runs first)."""

    def __init__(self):
        self.g = None

    def put(self, g):
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inst, ids, wemb, pemb, temb, gamma, beta, seed, p, meta):
        y, stats = ops().bert_embed_ln_fwd(inst, ids, wemb.detach(), pemb.detach(), temb.detach(), gamma.detach(),
                                           beta.detach(), seed, p)
        ctx.save_for_backward(inst, ids, wemb, pemb, temb, gamma, stats)
        ctx.cfg = (seed, p, meta)
        return y

    @staticmethod
    def backward(ctx, dy):
        inst, ids, wemb, pemb, temb, gamma, stats = ctx.saved_tensors
        seed, p, meta = ctx.cfg
        dx, slab = ops().bert_embed_ln_bwd(dy.contiguous(), inst, ids, wemb.detach(), pemb.detach(), temb.detach(),
                                           gamma.detach(), stats, seed, p, 0)
        S, L = inst.shape[0], ids.shape[1]
        HD = wemb.shape[1]
        rows = ids[inst.long()].reshape(-1).long()
        names = meta["names"]
        views = meta.get("grad_views")
        if views is not None and names["word"] in views:
            views[names["word"]].index_add_(0, rows, dx)
            dw = None
        else:
            dw = torch.zeros_like(wemb).index_add_(0, rows, dx) if wemb.requires_grad else None
        glue, maps = _glue_maps(meta, [names["gamma"], names["beta"], names["pos"], names["type"]])
        if glue is not None:   # all four as slab jobs of the step's one deterministic scatter-add
            glue.add(slab, glue.map_cat(maps[:2]), slab.shape[0])
            glue.add(dx.view(S, L * HD), maps[2][:L * HD], S)      # position rows 0 .. L-1
            glue.add(dx, maps[3][:HD], S * L)                        # token type 0
            return (None, None, dw, None, None, None, None, None, None, None)
        dpos_L = dx.view(S, L, HD).sum(0)
        dpos = torch.zeros_like(pemb)
        dpos[:L] = dpos_L
        dtype = torch.zeros_like(temb)
        dtype[0] = dpos_L.sum(0)
        sl = slab.sum(0)
        return (None, None, dw, _route_grad(meta, names["pos"], dpos), _route_grad(meta, names["type"], dtype),
                _route_grad(meta, names["gamma"], sl[0]), _route_grad(meta, names["beta"], sl[1]), None, None, None)


class _LnRes(torch.autograd.Function):
    """y = LN(res + dropout(a)); a = x W^T + ab (a _Linear with db_ext): ab's gradient is the column
    sum of da, which the backward kernel accumulates in the same pass (slab row 2)."""

    @staticmethod
    def forward(ctx, a, res, gamma, beta, seed, stream, p, meta, gname, bname, ab, abname, res_sink):
        """res_sink: a _ResGrad: the residual gradient goes to the dgrad GEMM of res's other consumer
        (returned as None here) instead of being summed by autograd."""
        y, stats = ops().bert_ln_res_fwd(a.contiguous(), res.contiguous(), gamma.detach(), beta.detach(), seed,
                                         stream, p)
        ctx.save_for_backward(a, res, gamma, stats)
        ctx.cfg = (seed, stream, p, meta, gname, bname, abname, res_sink)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, res, gamma, stats = ctx.saved_tensors
        seed, stream, p, meta, gname, bname, abname, res_sink = ctx.cfg
        dres, da, slab = ops().bert_ln_res_bwd(dy.contiguous(), a.contiguous(), res.contiguous(), gamma.detach(),
                                               stats, seed, stream, p, 0)
        if res_sink is not None:
            res_sink.put(dres)
            dres = None
        glue, maps = _glue_maps(meta, [gname, bname, abname])
        if glue is not None:   # [blocks][dgamma | dbeta | db] -> one slab job
            glue.add(slab, glue.map_cat(maps), slab.shape[0])
            return (da, dres, None, None, None, None, None, None, None, None, None, None, None)
        sl = slab.sum(0)
        return (da, dres, _route_grad(meta, gname, sl[0]), _route_grad(meta, bname, sl[1]), None, None, None, None,
                None, None, _route_grad(meta, abname, sl[2]), None, None)


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, meta, bname):
        y = ops().bert_bias_gelu_fwd(x.contiguous(), b.detach())
        ctx.save_for_backward(x, b)
        ctx.cfg = (meta, bname)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        meta, bname = ctx.cfg
        dx, slab = ops().bert_bias_gelu_bwd(dy.contiguous(), x, b.detach(), 0)
        glue, maps = _glue_maps(meta, [bname])
        if glue is not None:
            glue.add(slab, maps[0], slab.shape[0])
            return dx, None, None, None
        return dx, _route_grad(meta, bname, slab.sum(0)), None, None


class _Mha(torch.autograd.Function):
    """ctx = MHA(qkv), qkv = x Wqkv^T + [bq | bk | bv] (a _Linear with db_ext): the QKV bias gradient is
    the column sum of dqkv, accumulated by the backward kernel per (sequence, head) block."""

    @staticmethod
    def forward(ctx, qkv, inst, mask, L, nh, seed, stream, p, meta, bnames, bq, bk, bv):
        qkv = qkv.contiguous()
        out, lse = ops().bert_mha_fwd(qkv, inst, mask, L, nh, seed, stream, p)
        ctx.save_for_backward(qkv, out, lse, inst, mask)
        ctx.cfg = (L, nh, seed, stream, p, meta, bnames)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, inst, mask = ctx.saved_tensors
        L, nh, seed, stream, p, meta, bnames = ctx.cfg
        dqkv, bsum = ops().bert_mha_bwd(qkv, out, dout.contiguous(), lse, inst, mask, L, nh, seed, stream, p)
        glue, maps = _glue_maps(meta, bnames)
        if glue is not None:   # bsum [S][nh][3][64] -> q / k / v bias column (h, i, c) -> b_i[h * 64 + c]
            key = ("mha_bias", nh) + tuple(m.data_ptr() for m in maps)
            mp = glue._maps.get(key)
            if mp is None:
                mp = torch.stack([m.view(nh, 64) for m in maps], 1).reshape(-1).contiguous()
                glue._maps[key] = mp
            glue.add(bsum, mp, inst.shape[0])
            return (dqkv, None, None, None, None, None, None, None, None, None, None, None, None)
        db = bsum.view(inst.shape[0], nh, 3, 64).sum(0).transpose(0, 1).reshape(3, nh * 64)
        return (dqkv, None, None, None, None, None, None, None, None, None) + tuple(
            _route_grad(meta, bnames[i], db[i]) for i in range(3))


def layer_spans(model, flat_names, offsets, numels):
    """Flat-buffer (offset, numel) of each encoder layer's parameters (the DP overlap buckets)."""
    names = model.params.names()
    spans = []
    for i in range(model.cfg.bert_layers):
        pre = f"bert.encoder.layer.{i}."
        idx = [k for k, a in enumerate(flat_names) if names[a].startswith(pre)]
        spans.append((offsets[idx[0]], sum(numels[k] for k in idx)))
    return spans


def bert_encode(model, inst: torch.Tensor, data, training: bool, seed: int,
                grad_views: Optional[Dict[str, torch.Tensor]] = None, overlap=None, glue=None) -> torch.Tensor:
    """GPU BERT encoder + pooling + projection -> sentence vectors [S, bert_out_dim] fp32.
    ``overlap`` (parallel/dp.py::OverlapAllReduce over layer_spans) gets ``ready(i)`` when layer i's
    gradients are final, so DP all-reduces run under the rest of backward.  ``glue`` (ops/glue.py::StepGlue,
    trainer path): the LayerNorm / bias / embedding slab reductions are queued as slab jobs and scattered
    into the flat gradient by the glue's deterministic slab_scatter (one launch per 8 jobs) instead of a
    torch reduction + add per parameter (~190 launches per step); the caller flushes after backward."""
    cfg = model.cfg
    ids, mask, e1, e2 = data
    prm = model.params
    names = prm.names()                      # attr -> HF name
    by_name = {n: a for a, n in names.items()}
    P = lambda n: getattr(prm, by_name[n])  # noqa: E731
    S, L = inst.shape[0], ids.shape[1]
    Hd, nh, nl = cfg.bert_hidden, cfg.bert_heads, cfg.bert_layers
    pd = cfg.bert_dropout if training else 0.0
    pa = cfg.bert_attn_dropout if training else 0.0
    seed = int(seed) & 0x7FFFFFFF
    meta = {"grad_views": grad_views, "glue": glue if grad_views is not None else None}
    # ---- bf16 weight copy of all encoder layers: ONE cast of a contiguous flat-buffer region
    layer_names = [n for n in names.values() if n.startswith("bert.encoder.layer.")]
    lparams = [P(n) for n in layer_names]
    with torch.no_grad():
        region = _contiguous_region(lparams)
        wb = (region if region is not None else torch.cat([p.detach().reshape(-1) for p in lparams])).to(torch.bfloat16)
    offs, o = {}, 0
    for n, p in zip(layer_names, lparams):
        offs[n] = (o, p.numel())
        o += p.numel()

    def wspan(ns, shape):
        return wb.narrow(0, offs[ns[0]][0], sum(offs[m][1] for m in ns)).view(shape)

    def gspan(ns):
        """fp32 view of the flat gradient over consecutive params ns (trainer path) or None."""
        if grad_views is None:
            return None
        g0 = grad_views.get(by_name[ns[0]])
        if g0 is None:
            return None
        cnt = sum(offs[m][1] for m in ns)
        return torch.as_strided(g0, (cnt,), (1,), g0.storage_offset())

    def bias32(ns):
        """fp32 bias over consecutive params ns (the own NT GEMM's epilogue operand), detached."""
        ts = [P(n).detach() for n in ns]
        r = _contiguous_region(ts)
        return r if r is not None else torch.cat([t.reshape(-1) for t in ts])

    def linear(x, wn, bn, out_dim, in_dim, on_done=None, db_ext=False, dx_acc=None):
        Wb = wspan(wn, (out_dim, in_dim))
        bb = wspan(bn, (out_dim,)) if bn else None
        bf = bias32(bn) if bn and _own_nt() else None
        return _Linear.apply(x, Wb, bb, gspan(wn), gspan(bn) if bn else None, len(wn), on_done, db_ext, dx_acc, bf,
                             *[P(n) for n in wn], *[P(n) for n in (bn or [])])

    # DP overlap: the QKV projection's backward is the last backward op of layer i -> bucket i is final
    # (queued slab jobs of the layers above are scattered first: the bucket must hold final gradients)
    def _ready(i):
        def f():
            if meta["glue"] is not None:
                meta["glue"].flush()
            overlap.ready(i)
        return f
    layer_ready = _ready if overlap is not None else (lambda i: None)

    # ---- embeddings
    e = "bert.embeddings."
    emb_names = {"word": by_name[e + "word_embeddings.weight"], "pos": by_name[e + "position_embeddings.weight"],
                 "type": by_name[e + "token_type_embeddings.weight"], "gamma": by_name[e + "LayerNorm.weight"],
                 "beta": by_name[e + "LayerNorm.bias"]}
    x = _Embed.apply(inst, ids, P(e + "word_embeddings.weight"), P(e + "position_embeddings.weight"),
                     P(e + "token_type_embeddings.weight"), P(e + "LayerNorm.weight"), P(e + "LayerNorm.bias"),
                     seed, pd, dict(meta, names=emb_names))
    # ---- layers
    own_ffn = own_ffn_enabled(cfg.bert_intermediate, Hd)
    for i in range(nl):
        pre = f"bert.encoder.layer.{i}."
        a = pre + "attention."
        qn = [a + f"self.{k}.weight" for k in ("query", "key", "value")]
        bn = [a + f"self.{k}.bias" for k in ("query", "key", "value")]
        r1, r2 = _ResGrad(), _ResGrad()   # x feeds qkv + LN1's residual; x1 feeds FFN1 + LN2's residual
        qkv = linear(x, qn, bn, 3 * Hd, Hd, layer_ready(i), db_ext=True, dx_acc=r1)
        ctx = _Mha.apply(qkv, inst, mask, L, nh, seed, 17 + 3 * i, pa, meta, [by_name[n] for n in bn],
                         *[P(n) for n in bn])
        o = linear(ctx, [a + "output.dense.weight"], [a + "output.dense.bias"], Hd, Hd, db_ext=True)
        x = _LnRes.apply(o, x, P(a + "output.LayerNorm.weight"), P(a + "output.LayerNorm.bias"), seed, 18 + 3 * i, pd,
                         meta, by_name[a + "output.LayerNorm.weight"], by_name[a + "output.LayerNorm.bias"],
                         P(a + "output.dense.bias"), by_name[a + "output.dense.bias"], r1)
        I = cfg.bert_intermediate
        w1n, b1n, w2n, b2n = (pre + "intermediate.dense.weight", pre + "intermediate.dense.bias",
                              pre + "output.dense.weight", pre + "output.dense.bias")
        if own_ffn:
            o = _Ffn.apply(x, wspan([w1n], (I, Hd)), wspan([w2n], (Hd, I)), wspan([b2n], (Hd,)), gspan([w1n]),
                           gspan([w2n]), r2, meta, by_name[b1n], bias32([b2n]) if _own_nt() else None, P(w1n),
                           P(b1n), P(w2n))
        else:
            hpre = linear(x, [w1n], None, I, Hd, dx_acc=r2)
            h = _BiasGelu.apply(hpre, P(b1n), meta, by_name[b1n])
            o = linear(h, [w2n], [b2n], Hd, I, db_ext=True)
        x = _LnRes.apply(o, x, P(pre + "output.LayerNorm.weight"), P(pre + "output.LayerNorm.bias"), seed, 19 + 3 * i,
                         pd, meta, by_name[pre + "output.LayerNorm.weight"], by_name[pre + "output.LayerNorm.bias"],
                         P(pre + "output.dense.bias"), by_name[pre + "output.dense.bias"], r2)
    # ---- pooling + projection (fp32)
    xs = x.view(S, L, Hd)
    ar = torch.arange(S, device=x.device)
    if cfg.bert_pool == "entity":
        ie = inst.long()
        v = torch.cat([xs[ar, e1[ie].long()], xs[ar, e2[ie].long()]], -1)
    else:
        v = xs[:, 0]
    return torch.addmm(P("bert_proj/bias"), v.float(), P("bert_proj/kernel"))
