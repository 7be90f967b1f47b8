"""Sentence encoder on the GPU path: fused embedding + BiLSTM + self-attention pooling.

One ``torch.autograd.Function`` spans the whole encoder so that the bf16 BiLSTM output never
crosses an autograd boundary (its gradient stays fp32 inside ``backward``).

forward:  lstm_fwd (gather + MFMA recurrence, both directions; step records + dropout keep bits)
          ->  attention (MFMA projection, masked softmax, pooling)
backward: attention backward (recompute projection, dH premasked by the dropout keep bits, dW1/db1/dw2
          slabs)  ->  lstm_bwd (BPTT, dW/db/pos slabs)
ragged tiles (bf16 record path, default): rows are sorted by valid length (``ragged_plan``) and each
16-row tile's forward direction / attention stops at its longest length -- exact in parity mode;
``lstm_skip_padding`` adds TF sequence_length semantics for the backward direction.
bf16 (default): the attention kernels read the LSTM step records directly (rec_attn.hip; dH goes back
in lstm_bwd's lane layout); fp32 or fuse_rec_attn=False: natural-layout H rows + attn_fwd / attn_bwd.

Reference layers: model/base.py:76-86 (embedding), model/graph.py:30-53 (BiLSTM + attention),
model/layer_module.py:49-98 (self_attention).
"""
from __future__ import annotations

import os
import weakref

import torch

from ._ext import ops
from .packing import lstm_shape, pack_attn, pack_attn_rec, pack_lstm


def _route_grad(meta, name, g):
    """Write a parameter gradient straight into the flat gradient buffer when the trainer provides
    its view (``meta['grad_views']``): no AccumulateGrad add kernel, no extra copy."""
    views = meta.get("grad_views")
    if g is None:
        return None
    if views is not None and name in views:
        views[name].add_(g.reshape(views[name].shape))
        return None
    return g.contiguous()


_WROWS: dict = {}
_QI = [0, 4, 1, 5, 2, 6, 3, 7]   # word_rows column order (feature q, q + 4 per lane group q)


DIRECT_X_CALLS = [0]   # forwards that ran direct x (tests assert the path engaged)


def direct_x_enabled() -> bool:
    """Direct-x recurrences (lstm.hip xd_build): INA_DIRECT_X=0 keeps the x_gather record (A/B, tests)."""
    return os.environ.get("INA_DIRECT_X", "1") != "0"


def word_rows(word: torch.Tensor, wemb: torch.Tensor, fresh: bool):
    """Word-table rows per dataset token, bf16 [NI * L, 8] (zero padded; the gate MFMAs take x in bf16
    anyway), for lstm_fwd's x gather: one 16-byte load per token from a per-instance contiguous run
    instead of a random row of the 400k-row table.  Columns are q-interleaved, [f0 f4 f1 f5 f2 f6 f3 f7]:
    the recurrences' lane group q holds features q and q + 4, ONE dword at byte 4q (direct x, lstm.hip).
    A frozen table (the reference default, model/base.py:55-59) is gathered once per (ids, table
    version); ``fresh`` (trained word table, updated in place by the fused optimizer) gathers every
    step.  None for word vectors wider than 8 (the kernel then gathers from the table itself)."""
    if wemb.shape[1] > 8:
        return None
    # keyed by tensor identity (weak references), not data_ptr: a freed tensor's address is reused
    # by the caching allocator, and a data_ptr key would then hand back another table's rows
    key = (id(word), id(wemb), wemb._version)
    if not fresh:
        hit = _WROWS.get(key)
        if hit is not None and hit[0]() is word and hit[1]() is wemb:
            return hit[2]
    E = wemb.shape[1]
    rows = torch.nn.functional.pad(wemb.detach().float().index_select(0, word.reshape(-1).long()), (0, 8 - E))
    rows = rows[:, _QI].to(torch.bfloat16).contiguous()
    if not fresh:
        if len(_WROWS) >= 4:
            _WROWS.pop(next(iter(_WROWS)))
        _WROWS[key] = (weakref.ref(word), weakref.ref(wemb), rows)
    return rows


RAGGED_MIN_ROWS = 16384   # 1024 tiles: ~4 per CU


def ragged_plan(inst: torch.Tensor, lengths: torch.Tensor, skip: bool, L: int = 64):
    """Length-sorted rows for the record kernels: (inst_sorted, perm, tlen, slen).

    perm = the stable argsort of the rows' valid lengths (row s of every record array is row perm[s] of
    e / alphas / de); tlen [tiles] = each 16-row tile's longest length (>= 1): the forward direction and
    the attention stop there -- padding outputs are masked out of the attention (alpha exactly 0), so
    this is exact -- and sorted tiles make it ~the rows' own lengths.  slen (lstm_skip_padding only) =
    the sorted lengths, for the backward direction's per-row sequence_length resets."""
    S = inst.shape[0]
    if inst.is_cuda and inst.dtype == torch.int32 and lengths.dtype == torch.int32:
        # one counting-sort pass on the device (csrc/kernels/ragged.hip): lengths are 0..L
        inst_s, perm, tlen, slen = ops().ragged_sort(inst.contiguous(), lengths.contiguous(), L)
        return inst_s, perm, tlen, (slen if skip else None)
    lens = lengths.index_select(0, inst.long())
    perm = torch.argsort(lens, stable=True)
    slen = lens.index_select(0, perm)
    ntiles = (S + 15) // 16
    last = torch.clamp(torch.arange(ntiles, device=inst.device) * 16 + 15, max=max(S - 1, 0))
    tlen = torch.clamp(slen.index_select(0, last), min=1).to(torch.int32).contiguous()
    return (inst.index_select(0, perm).contiguous(), perm.to(torch.int32).contiguous(), tlen,
            slen.to(torch.int32).contiguous() if skip else None)


class EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inst, word, pos1, pos2, mask, wemb, p1emb, p2emb, Kf, bf, Kb, bb, W1, b1, w2, meta):
        """meta = dict(U, bf16, keep_prob, seed, word_grad, lstm_blocks, attn_blocks)."""
        o = ops()
        U, bf16 = meta["U"], meta["bf16"]
        DIN = wemb.shape[1] + 2 * p1emb.shape[1]
        sh = lstm_shape(U, DIN, bf16)
        pk = meta.get("packs")
        if pk is not None:   # StepGlue: every pack of the step came from one gather launch
            apack, a2pack, bias = pk["apack"], pk["a2pack"], pk["bias2"]
        else:
            apack, a2pack = pack_lstm(Kf, Kb, U, DIN, bf16)
            bias = torch.stack([bf.detach(), bb.detach()]).float().contiguous()
        # (ctx.needs_input_grad is True for trainable parameters even under torch.no_grad(): the caller
        # passes the grad mode, so eval / serving runs the forward without the backward's stash)
        need_grad = meta.get("need_grad")
        if need_grad is None:
            need_grad = ctx.needs_input_grad[5:15].count(True) > 0 if hasattr(ctx, "needs_input_grad") else True
        kp = float(meta["keep_prob"])
        lstm_args = (inst, word, pos1, pos2, wemb.detach().contiguous(), p1emb.detach().contiguous(),
                     p2emb.detach().contiguous(), apack, bias, U, sh["NX"])
        wrows = word_rows(word, wemb, bool(meta.get("word_grad", False))) if bf16 else None
        tail = (int(meta["seed"]), kp, meta.get("seed_dev"), wrows)
        b1c, w2c = b1.detach().contiguous(), w2.detach().reshape(-1).contiguous()
        rec = bf16 and meta.get("fuse_rec_attn", True) and o.rec_attn_ok(U, word.shape[1])
        skip = bool(meta.get("skip_padding", False))
        lengths = meta.get("lengths")
        if skip and not (rec and lengths is not None):
            raise NotImplementedError("lstm_skip_padding on the GPU needs the bf16 record path (u in {8, 20, 32}, "
                                      "L <= 64) and device lengths")
        perm = tlen = slen = None
        # direct x: the recurrences read the word rows + LDS position tables (shifted ids), no xg record.  It
        # pays once the kernels are throughput-bound (same row threshold as the ragged tiles): 1,616,764 vs
        # 1,588,243 episodes/s at 2048 episodes, 3,543 vs 3,569 at 1 episode (profiles/r4_direct_x/small)
        direct = (rec and wrows is not None and sh["NX"] == 4 and bool(meta.get("pos_shift", False))
                  and direct_x_enabled() and inst.shape[0] >= meta.get("direct_x_min_rows", RAGGED_MIN_ROWS))
        DIRECT_X_CALLS[0] += int(direct)
        if rec:
            # attention straight from the step records (no natural-layout copy of H)
            w1pack, w1tpack = ((pk["w1rpack"], pk["w1rtpack"]) if pk is not None and "w1rpack" in pk
                               else pack_attn_rec(W1))
            # ragged tiles pay off once the kernels are throughput-bound (many tiles per CU); small steps are
            # latency-bound on the backward direction's full-length chain and would only add the sort
            if lengths is not None and (skip or (meta.get("ragged", True)
                                                 and inst.shape[0] >= meta.get("ragged_min_rows", RAGGED_MIN_ROWS))):
                inst, perm, tlen, slen = ragged_plan(inst, lengths, skip, int(word.shape[1]))
                lstm_args = (inst,) + lstm_args[1:]
            hlane, cst, hnat, dmask, xg, e, alphas = o.lstm_attn_fwd(*lstm_args, bool(need_grad), *tail,
                                                                     mask, w1pack, b1c, w2c, tlen, perm, slen,
                                                                     direct)
        else:
            w1pack, w1tpack = (pk["w1pack"], pk["w1tpack"]) if pk is not None else pack_attn(W1, bf16)
            hlane, cst, hnat, dmask, xg = o.lstm_fwd(*lstm_args, bf16, bool(need_grad), *tail)
            e, alphas = o.attn_fwd(hnat, inst, mask, w1pack, b1c, w2c, U, bf16, int(meta.get("attn_blocks", 0)))
        if need_grad:
            ctx.save_for_backward(inst, word, pos1, pos2, wemb, p1emb, p2emb, apack, a2pack, bias, hlane, cst,
                                  w1pack, w1tpack, b1, w2, alphas, hnat, dmask, xg, e, perm, tlen, slen,
                                  wrows if direct else None)
            ctx.meta = dict(meta, NX=sh["NX"], DIN=DIN, rec=rec)
        ctx.mark_non_differentiable(alphas)
        ctx.set_materialize_grads(False)   # no zero-fill launch for the alphas gradient
        return e, alphas

    @staticmethod
    def backward(ctx, de, _dalpha):
        o = ops()
        (inst, word, pos1, pos2, wemb, p1emb, p2emb, apack, a2pack, bias, hlane, cst, w1pack, w1tpack, b1, w2,
         alphas, hnat, dmask, xg, e, perm, tlen, slen, wrows) = ctx.saved_tensors
        m = ctx.meta
        U, bf16, DIN = m["U"], m["bf16"], m["DIN"]
        H2 = 2 * U
        b1c, w2c = b1.detach().contiguous(), w2.detach().reshape(-1).contiguous()
        word_grad = bool(m.get("word_grad", False))
        if m["rec"]:   # dH in lstm_bwd's lane layout [tiles, 2, L, U/4, 64]
            dH, aslab = o.rec_attn_bwd(hlane, dmask, w1pack, w1tpack, b1c, w2c, de.contiguous().float(), e, alphas,
                                       U, float(m["keep_prob"]), int(m.get("attn_blocks", 0)), tlen, perm)
        else:
            dH, aslab = o.attn_bwd(hnat, inst, w1pack, w1tpack, b1c, w2c, de.contiguous().float(), alphas, U, bf16,
                                   int(m.get("attn_blocks", 0)))
        dw_slab, dpos_slab, dwemb = o.lstm_bwd(inst, word, pos1, pos2, wemb.detach().contiguous(),
                                               p1emb.detach().contiguous(), p2emb.detach().contiguous(), apack, a2pack,
                                               bias, hlane, cst, dH, dmask, xg, U, m["NX"], bf16, word_grad,
                                               int(m.get("lstm_blocks", 0)), int(m["seed"]), float(m["keep_prob"]),
                                               bool(m.get("pos_shift", False)), tlen, slen, wrows)
        return EncoderFn._grads(ctx, m, aslab, dw_slab, dpos_slab, dwemb)

    @staticmethod
    def _grads(ctx, m, aslab, dw_slab, dpos_slab, dwemb):
        """Slabs -> parameter gradients.  aslab: [blocks, 2U*2U + 2*2U] (attention kernels)."""
        word, p1emb, p2emb = ctx.saved_tensors[1], ctx.saved_tensors[5], ctx.saved_tensors[6]
        U, DIN = m["U"], m["DIN"]
        H2 = 2 * U
        word_grad = bool(m.get("word_grad", False))
        glue = m.get("glue")
        if glue is not None:
            # slabs -> flat gradient in the step's single slab_scatter_add launch (StepGlue.flush)
            p = m["pdict"]
            glue.add(aslab, glue.map_attn(p, H2), aslab.shape[0])
            glue.add(dw_slab, glue.map_lstm_dw(p, U, DIN), dw_slab.shape[0])
            L, PD = word.shape[1], p1emb.shape[1]
            mp = glue.map_pos(p, L, PD)
            glue.add(dpos_slab, mp, dpos_slab.numel() // mp.numel())
            wg = _route_grad(m, "word_embedding", dwemb) if word_grad else None
            return (None,) * 5 + (wg,) + (None,) * 10
        a = aslab.sum(0)
        dW1 = a[: H2 * H2].view(H2, H2)
        db1 = a[H2 * H2: H2 * H2 + H2]
        dw2 = a[H2 * H2 + H2:].view(H2, 1)
        D = dw_slab.sum(0)                         # [2, 4U, DIN+U+1]
        dKf = D[0, :, : DIN + U].t()
        dKb = D[1, :, : DIN + U].t()
        dbf = D[0, :, DIN + U]
        dbb = D[1, :, DIN + U]
        P = dpos_slab.sum((0, 1))                  # [2 tables, 2L, PD]
        dp1 = P[0][: p1emb.shape[0]]
        dp2 = P[1][: p2emb.shape[0]]
        grads = dict(word_embedding=dwemb if word_grad else None, pos1_embedding=dp1, pos2_embedding=dp2,
                     lstm_fw_kernel=dKf, lstm_fw_bias=dbf, lstm_bw_kernel=dKb, lstm_bw_bias=dbb, attn_kernel=dW1,
                     attn_bias=db1, attn_w2=dw2)
        order = ("word_embedding", "pos1_embedding", "pos2_embedding", "lstm_fw_kernel", "lstm_fw_bias",
                 "lstm_bw_kernel", "lstm_bw_bias", "attn_kernel", "attn_bias", "attn_w2")
        return (None, None, None, None, None) + tuple(_route_grad(m, k, grads[k]) for k in order) + (None,)


def encode(inst, data, params, meta):
    """data = (word, pos1, pos2, mask) device int32 arrays [NI, L]; returns (e [S, 2u], alphas [S, L])."""
    word, pos1, pos2, mask = data
    # position ids known to be shifted aranges (ops/sampler.py::DeviceArrays): cheaper pos-table gradient
    meta = dict(meta, pos_shift=bool(getattr(data, "pos_shift", False)), lengths=getattr(data, "lengths", None),
                need_grad=torch.is_grad_enabled() and any(
                    isinstance(t, torch.Tensor) and t.requires_grad for t in params.values()))
    return EncoderFn.apply(inst, word, pos1, pos2, mask, params["word_embedding"], params["pos1_embedding"],
                           params["pos2_embedding"], params["lstm_fw_kernel"], params["lstm_fw_bias"],
                           params["lstm_bw_kernel"], params["lstm_bw_bias"], params["attn_kernel"],
                           params["attn_bias"], params["attn_w2"], meta)
