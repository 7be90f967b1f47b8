"""Wide-layer GPU path: BiLSTM with per-step hipBLASLt GEMMs + fused HIP cell kernels, attention /
routing / NTN as batched GEMM formulations (the reference's paper configuration u=128, E=300 and any
shape outside the fused kernels' instantiations).

BiLSTM (both directions batched; reference model/graph.py:34-49):
    Gx = X W_x + b          one GEMM over all S*L tokens per direction          (hipBLASLt, bf16)
    per step: Gh = h W_h    one batched GEMM over the two directions, fp32 out  (hipBLASLt)
              ina.lstm_wide_fwd_step: activations, c/h update, dropout output   (HIP, fused)
    backward per step: ina.lstm_wide_bwd_step (dG), dh_rec = dG W_h^T (GEMM);
    then dW_h = H_prev^T dG, dW_x = X^T dG, dX = dG W_x^T as whole-sequence GEMMs (split-K).
Attention / routing / NTN at wide H use the GEMM formulations of models/reference.py (the NTN as
the two GEMMs of SURVEY K7 -- P = C M, then batched P Q^T) under autograd.
"""
from __future__ import annotations

import weakref

import numpy as np
import torch

from ._ext import ops


def _own_tn_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Operands the own TN split-K GEMM takes (csrc/kernels/gemm.hip): bf16 GPU rows, unit column stride, widths and
    row strides multiples of 8.  INA_WIDE_OWN_WGRAD=0 selects hipBLASLt (A/B)."""
    import os
    return (os.environ.get("INA_WIDE_OWN_WGRAD", "1") != "0" and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
            and a.stride(1) == 1 and b.stride(1) == 1 and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.shape[0] > 0)


def _wgrad_parts(a: torch.Tensor, b: torch.Tensor, split: int = 16, own: bool = True):
    """(partials [ns, m, n] fp32, ns) of a^T b, summed by _wgrad or by the step glue's ordered slab reduction."""
    if own and _own_tn_ok(a, b):
        part = ops().gemm_wgrad(a, b, 0)
        return part, part.shape[0]
    T = a.shape[0]
    sp = split
    while sp > 1 and (T % sp or T < 256 * sp):
        sp //= 2
    if sp > 1:
        return torch.bmm(a.view(sp, T // sp, -1).transpose(1, 2), b.view(sp, T // sp, -1), out_dtype=torch.float32), sp
    return torch.mm(a.t(), b, out_dtype=torch.float32).unsqueeze(0), 1


def _wgrad(a: torch.Tensor, b: torch.Tensor, split: int = 16, own: bool = True) -> torch.Tensor:
    """a^T b in fp32 for tall bf16 a [T, m], b [T, n]: the own TN split-K GEMM (one round of 256 x 256 output tiles
    over the CUs, fp32 slabs + an ordered sum; 242 vs 245 us for hipBLASLt's split-128 batch at the paper
    attention dW1, profiles/r6_gemm) or, for other operands, hipBLASLt with K = T split into `split` chunks
    (a single K = 1.2 M GEMM runs on a handful of output tiles; a T that `split` does not divide takes the largest
    smaller power-of-two split that does)."""
    part, ns = _wgrad_parts(a, b, split, own)
    return part.sum(0) if ns > 1 else part[0]


class WideBiLSTM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Kf, bf, Kb, bb, U, seed, keep_prob):
        """X [S, L, D] bf16 or fp32 (gathered embeddings) -> dropout output [S, L, 2U] bf16."""
        o = ops()
        S, L, D = X.shape
        dev = X.device
        Wx = torch.stack([Kf[:D], Kb[:D]]).detach().to(torch.bfloat16)            # [2, D, 4U]
        Wh = torch.stack([Kf[D:], Kb[D:]]).detach().to(torch.bfloat16)            # [2, U, 4U]
        b = torch.stack([bf, bb]).detach().float()                                # [2, 4U]
        Xb = X.detach().reshape(S * L, D).to(torch.bfloat16)
        # both directions' input projections as ONE batched GEMM straight into [2, S*L, 4U] fp32, bias
        # added in place (a per-direction mm + add + stack moved ~10 GB more per step at u=128)
        gx = torch.bmm(Xb.unsqueeze(0).expand(2, -1, -1), Wx, out_dtype=torch.float32)
        gx += b.unsqueeze(1)
        gx = gx.view(2, S, L, 4 * U)
        need = ctx.needs_input_grad[0] or any(ctx.needs_input_grad[1:5])
        c = torch.zeros(2, S, U, device=dev)
        hcur = torch.zeros(2, S, U, device=dev, dtype=torch.bfloat16)
        hall = torch.empty(2, S, L, U, device=dev, dtype=torch.bfloat16)
        call = torch.empty(2, S, L, U, device=dev) if need else torch.empty(0, device=dev)
        acts = (torch.empty(2, S, L, 4 * U, device=dev, dtype=torch.bfloat16) if need
                else torch.empty(0, device=dev, dtype=torch.bfloat16))
        hout = torch.empty(S, L, 2 * U, device=dev, dtype=torch.bfloat16)
        for tau in range(L):
            gh = torch.bmm(hcur, Wh, out_dtype=torch.float32)
            o.lstm_wide_fwd_step(gx, gh, c, hcur, hall, call, acts, hout, tau, int(seed), float(keep_prob))
        if need:
            ctx.save_for_backward(Xb, Wx, Wh, hall, call, acts)
            ctx.cfg = (S, L, D, U, int(seed), float(keep_prob))
            ctx.xdtype = X.dtype
        return hout

    @staticmethod
    def backward(ctx, dout):
        o = ops()
        Xb, Wx, Wh, hall, call, acts = ctx.saved_tensors
        S, L, D, U, seed, kp = ctx.cfg
        dev = Xb.device
        dH = dout.contiguous().to(torch.bfloat16)
        dhrec = torch.zeros(2, S, U, device=dev)
        dcrec = torch.zeros(2, S, U, device=dev)
        dG = torch.empty(2, S, L, 4 * U, device=dev, dtype=torch.bfloat16)
        nodg = torch.empty(0, device=dev, dtype=torch.bfloat16)
        WhT = Wh.transpose(1, 2).contiguous()                                    # [2, 4U, U]
        G4 = 4 * U
        for tau in reversed(range(L)):
            o.lstm_wide_bwd_step(dH, dhrec, dcrec, call, acts, dG, nodg, tau, seed, kp)
            if tau > 0:
                # this step's dG rows of both directions (times tau and L-1-tau) read in place: one
                # strided view (batch stride S*L*4U + (t1 - t0)*4U, row stride L*4U), no per-step copy
                t0, t1 = tau, L - 1 - tau
                cur = dG.as_strided((2, S, G4), (S * L * G4 + (t1 - t0) * G4, L * G4, 1), t0 * G4)
                dhrec = torch.bmm(cur, WhT, out_dtype=torch.float32)
        # h_{t-1} in each direction's processing order (zeros at its first step)
        hprev = torch.zeros_like(hall)
        hprev[0, :, 1:] = hall[0, :, :-1]
        hprev[1, :, :-1] = hall[1, :, 1:]
        dKs, dbs = [], []
        dX = None
        for d in range(2):
            g = dG[d].reshape(S * L, 4 * U)
            dWx = _wgrad(Xb, g)
            dWh = _wgrad(hprev[d].reshape(S * L, U), g)
            dKs.append(torch.cat([dWx, dWh], 0))
            dbs.append(g.sum(0, dtype=torch.float32))
            dx = torch.mm(g, Wx[d].t(), out_dtype=torch.float32)
            dX = dx if dX is None else dX + dx
        return dX.view(S, L, D).to(ctx.xdtype), dKs[0], dbs[0], dKs[1], dbs[1], None, None, None


_WTAB: dict = {}


def word_table_bf16(wemb: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a FROZEN word table, cached per (tensor, version): the x rows enter the GEMM as bf16
    anyway, and the wide gather's random row reads are ~2/3 of its traffic at 300-d words.  An in-place
    update of the table bumps its version counter and refreshes the copy.  Keyed by tensor identity (a
    weak reference), not data_ptr: a freed table's address is reused by the caching allocator, and a
    same-shape table allocated there at version 0 would otherwise get the old table's rows."""
    key = (id(wemb), wemb._version)
    ent = _WTAB.get(key)
    if ent is not None and ent[0]() is wemb:
        return ent[1]
    if len(_WTAB) >= 2:
        _WTAB.pop(next(iter(_WTAB)))
    tab = wemb.detach().to(torch.bfloat16).contiguous()
    _WTAB[key] = (weakref.ref(wemb), tab)
    return tab


def x_projection(Xb: torch.Tensor, pk: dict) -> torch.Tensor:
    """Xb [T, DP] x wxc [DP, 2 G4] -> bf16 [T, 2 G4] on the own GEMM (csrc/kernels/gemm.hip; its widened
    16-byte epilogue stores: 1.12 ms against hipBLASLt's 1.23 ms at the paper configuration,
    profiles/r5_widen) where its limits hold (N % 256, K % 64, 32-bit operand offsets), else hipBLASLt."""
    M, K = Xb.shape
    wt = pk.get("wxcT")
    lda = Xb.stride(0)
    if (wt is not None and wt.shape[0] % 256 == 0 and K % 64 == 0 and Xb.stride(1) == 1 and lda % 8 == 0
            and M * lda * 2 < (1 << 31)):
        return ops().bert_gemm(Xb, wt, None, None, 0)[0]   # (Xb may be the x columns of wider rows)
    return torch.mm(Xb, pk["wxc"])


class WideSeqBiLSTM(torch.autograd.Function):
    """Embedding + BiLSTM of the wide path on hand-written kernels (lstm_wide.hip, U in {64, 100, 128}):
      wide_x_gather     the encoder input rows Xb [S*L, DP] bf16 in one pass (E + 2PD embedding columns,
                        a ones column, zero padding: packing.wide_x_cols);
      one GEMM          x W_x for both directions side by side (permuted, pre-scaled gate columns, bf16
                        out, [S*L, 2 G4]);
      lstm_wide_seq_fwd the whole forward recurrence in ONE launch (W_h in registers, h through LDS,
                        fused bias / activations / DropoutWrapper output);
      lstm_wide_seq_bwd the whole BPTT in one launch (dG stash); weight gradients as whole-sequence
                        GEMMs; the input gradient only for the trainable columns (the reference's word table
                        is frozen, model/base.py:55-59) and the position tables' gradient by
                        wide_pos_grad (FewRel's shifted-arange position ids) or a one-hot GEMM."""

    @staticmethod
    def forward(ctx, inst, word, pos1, pos2, wemb, p1emb, p2emb, Kf, bf, Kb, bb, U, seed, keep_prob, pos_shift,
                packs=None, gl=None):
        from .packing import pack_lstm_wide
        o = ops()
        S, L = inst.shape[0], word.shape[1]
        E, P = wemb.shape[1], p1emb.shape[1]
        D = E + 2 * P
        pk = packs if packs is not None else pack_lstm_wide(Kf, bf, Kb, bb, U, D)
        wtab = word_table_bf16(wemb) if not wemb.requires_grad else wemb.detach().float().contiguous()
        need = any(ctx.needs_input_grad[4:11])
        UP = (U + 31) // 32 * 32
        DP = (D + 1 + 31) // 32 * 32
        # training: each x row is followed by the two directions' h_{t-1} stash columns (written by the forward
        # kernel), so ONE split-K GEMM over [x | h_fw | h_bw] rows gives dW_x, db and both dW_h reading dG once
        # (1,385 vs 1,506 us for the three GEMMs at the paper configuration, a round-5 probe, profiles/r5_merged)
        Xw = o.wide_x_gather(inst, word, pos1, pos2, wtab, p1emb.detach().float().contiguous(),
                             p2emb.detach().float().contiguous(), 2 * UP if need else 0)
        Xb = Xw[:, :DP]
        # x W_x for both directions as ONE bf16-output GEMM (the kernel adds the fp32 biases): an fp32 output
        # plus a separate bias pass moved ~15 GB per step at the paper configuration
        gx = x_projection(Xb, pk)
        hout, _, acts, cst = o.lstm_wide_seq_fwd(gx, pk["bx"], pk["apk"], S, L, U, bool(need), int(seed),
                                                 float(keep_prob), Xw if need else Xw.new_empty(0), DP)
        if need:
            ctx.save_for_backward(inst, word, pos1, pos2, Xw, pk["wxtc"], pk["a2pk"], acts, cst)
            ctx.cfg = (S, L, E, P, U, int(seed), float(keep_prob), bool(pos_shift), p1emb.shape[0], wemb.shape[0])
            # gl = (StepGlue, params): the gradients go to the glue's single scatter-add into the flat gradient (no
            # .sum(0) of the split-K partials, no unpack gather, no autograd accumulation adds)
            ctx.gl = gl
        return hout

    @staticmethod
    def backward(ctx, dout):
        from .packing import unpack_merged_wgrad
        o = ops()
        inst, word, pos1, pos2, Xw, wxtc, a2pk, acts, cst = ctx.saved_tensors
        S, L, E, P, U, seed, kp, shift, P2, V = ctx.cfg
        D = E + 2 * P
        need_w = ctx.needs_input_grad[4]
        # the position columns of the input gradient straight from the BPTT kernel (dG W_pos^T on the LDS
        # image of each step's dG); the word columns only for a trainable word table, as a GEMM
        fuse = not need_w and 2 * P <= 16
        wpk = pos_frags(wxtc, E, D) if fuse else wxtc.new_empty(0)
        dG, dxpd = o.lstm_wide_seq_bwd(dout.contiguous().to(torch.bfloat16), acts, cst, a2pk, S, L, U, seed, kp,
                                       wpk, 2 * P)
        G4 = dG.shape[1] // 2
        UP = G4 // 4
        DP = Xw.shape[1] - 2 * UP
        # ONE GEMM for both directions' x- and h-kernel gradients over the rows [x | h_fw | h_bw] (the two
        # cross-direction blocks h_fw^T dG_bw / h_bw^T dG_fw are computed and dropped: 12% more FLOPs, dG read
        # once); x's ones column (row D) makes it the bias gradient as well
        # [DP + 2 UP, 2 G4] on hipBLASLt split-64: 1,227 us in the step (profiles/r5_merged); the own TN kernel on the
        # 512 rows that fill 256-row tiles + gemm_tn.hip for the 64-row h_bw tail took 1,190 + 224 us (paper 32.2-32.6k
        # vs 32.9-33.1k episodes/s, profiles/r6_paper1): at this shape hipBLASLt's main loop (1.14 PF/s) beats the own
        # one (1.04)
        gl = ctx.gl if not need_w else None
        if gl is not None:
            glue, p = gl
            part, ns = _wgrad_parts(Xw, dG, 64, own=False)
            glue.add(part, glue.map_merged_lstm(p, U, D, DP, G4), ns)
            dKs, dbs = [None, None], [None, None]
        else:
            dwall = _wgrad(Xw, dG, 64, own=False)
            dKs, dbs = unpack_merged_wgrad(dwall, U, D)                  # both directions, one gather
        if fuse:
            dxp = dxpd                                                    # [2, S*L, 2P]: per direction
        else:
            cols = slice(0, D) if need_w else slice(E, D)
            dX = torch.mm(dG, wxtc[cols].t(), out_dtype=torch.float32)  # both directions: K = 2 G4
            dxp = dX[:, -2 * P:].contiguous()
        if shift:
            tp = o.wide_pos_grad(dxp, inst, pos1, pos2, P2)             # sums the direction planes
            dp1, dp2 = tp[0], tp[1]
            if gl is not None:
                glue.add(tp, glue.map_cat([glue.map_identity(p["pos1_embedding"]),
                                           glue.map_identity(p["pos2_embedding"])]), 1)
                dp1 = dp2 = None
        else:
            if dxp.dim() == 3:
                dxp = dxp.sum(0)
            il = inst.long()
            dp1 = table_grad(pos1[il].reshape(-1).long(), dxp[:, :P], P2)
            dp2 = table_grad(pos2[il].reshape(-1).long(), dxp[:, P:], P2)
        dw = None
        if need_w:
            dw = table_grad(word[inst.long()].reshape(-1).long(), dX[:, :E], V)
        return (None, None, None, None, dw, dp1, dp2, dKs[0], dbs[0], dKs[1], dbs[1], None, None, None, None, None,
                None)


def pos_frags(wxtc: torch.Tensor, E: int, D: int) -> torch.Tensor:
    """MFMA A fragments of W_pos^T for the BPTT kernel's fused dX_pos (csrc/kernels/lstm_wide.hip): rows
    E .. D of wxtc [D, 2 G4] (the position columns' x-projection weights, permuted gate columns, unscaled)
    zero-padded to 16 rows -> [2 dirs][G4 / 32 K-steps][64 lanes][8] bf16, lane = 16 q + n holding row n,
    gate columns 32 ks + 8 q .. + 8 of its direction."""
    G4 = wxtc.shape[1] // 2
    wp = torch.nn.functional.pad(wxtc[E:D], (0, 0, 0, 16 - (D - E)))                # [16, 2 G4]
    return wp.view(16, 2, G4 // 32, 4, 8).permute(1, 2, 3, 0, 4).contiguous().to(torch.bfloat16)


def table_grad(idx: torch.Tensor, d: torch.Tensor, rows: int) -> torch.Tensor:
    """sum of the rows d[i] into table row idx[i] -- deterministic: a one-hot GEMM, split-K for small tables
    (autograd's index backward is a sort + segmented accumulate, 14 ms per [74, 5] table per step at the
    paper configuration); index_add_ for large tables (trained word embeddings)."""
    if rows > 4096:
        return torch.zeros(rows, d.shape[1], device=d.device, dtype=torch.float32).index_add_(0, idx, d.float())
    fd = d.float()
    T, C = fd.shape
    nb = SmallTableGather.SPLIT
    Tp = (T + nb - 1) // nb * nb
    fi = idx
    if Tp != T:   # pad with tokens of zero gradient
        fi = torch.cat([fi, fi.new_zeros(Tp - T)])
        fd = torch.cat([fd, fd.new_zeros(Tp - T, C)])
    oh = torch.nn.functional.one_hot(fi, rows).to(torch.float32).view(nb, Tp // nb, rows)
    return torch.bmm(oh.transpose(1, 2), fd.view(nb, Tp // nb, C)).sum(0)


class SmallTableGather(torch.autograd.Function):
    """rows = table[idx] for a SMALL table (the [2L, 5] position tables).  Autograd's index backward
    scatters 1.2 M token gradients into ~74 rows with a sort + segmented accumulate that measured
    14.4 ms per table per step at the paper configuration (41% of the step, profiles/r2_paper1);
    here the table gradient is the GEMM OneHot(idx)^T dRows in fp32, in token chunks (deterministic,
    a few hundred microseconds)."""

    SPLIT = 256   # split-K batches: a [P, T] x [T, 5] GEMM has ~5 output tiles (measured 0.5 ms per
                  # 2^18-token chunk as one GEMM); as 256 independent K-slices + an ordered sum it fills the chip

    @staticmethod
    def forward(ctx, table, idx):
        ctx.save_for_backward(idx)
        ctx.rows = table.shape[0]
        return table[idx]

    @staticmethod
    def backward(ctx, d):
        (idx,) = ctx.saved_tensors
        fi = idx.reshape(-1)
        return table_grad(fi, d.reshape(fi.shape[0], -1), ctx.rows).to(d.dtype), None


class ProjBF16(torch.autograd.Function):
    """Z = X W in fp32 from bf16 operands (X [T, n] bf16, W [n, m] fp32 master): the attention
    projection of the wide path as a bf16 MFMA GEMM (the fp32 formulation of models/reference.py ran
    it as an fp32 GEMM over all S*L tokens).  Backward: dX = dZ W^T (bf16), dW = X^T dZ (fp32)."""

    @staticmethod
    def forward(ctx, X, W):
        Wb = W.detach().to(torch.bfloat16)
        ctx.save_for_backward(X, Wb)
        return torch.mm(X, Wb, out_dtype=torch.float32)

    @staticmethod
    def backward(ctx, dZ):
        X, Wb = ctx.saved_tensors
        dZb = dZ.contiguous().to(torch.bfloat16)
        dX = torch.mm(dZb, Wb.t()) if ctx.needs_input_grad[0] else None
        dW = _wgrad(X, dZb) if ctx.needs_input_grad[1] else None
        return dX, dW


class WideAttn(torch.autograd.Function):
    """Fused self-attention pooling (csrc/kernels/attn_wide.hip; reference model/layer_module.py:49-98)
    over the bf16 BiLSTM output Hb [S, L, H], H = 2u in {128, 200, 256}: one forward kernel (projection
    on MFMA, tanh / score / masked softmax / pooling on the staged block), one backward kernel (dH,
    the dZ operand and dw2 / db1 partials) + the dW1 = H^T dZ split-K GEMM.  alphas carry no
    gradient (the reference fetches them for inspection only, model/base.py:144)."""

    @staticmethod
    def forward(ctx, Hb, inst, mask, W1, b1, w2, packs=None, gl=None):
        from .packing import pack_attn_wide
        pk = packs if packs is not None else pack_attn_wide(W1, b1, w2)
        e, alpha = ops().wide_attn_fwd(Hb, inst, mask, pk["w1t"], pk["b1"], pk["w2"])
        ctx.save_for_backward(Hb, inst, mask, alpha)
        ctx.pk = pk
        ctx.gl = gl   # (StepGlue, params): gradients into the glue (see WideSeqBiLSTM)
        ctx.mark_non_differentiable(alpha)
        return e, alpha

    @staticmethod
    def backward(ctx, de, _dalpha):
        Hb, inst, mask, alpha = ctx.saved_tensors
        pk = ctx.pk
        H = Hb.shape[-1]
        dH, dZ, part = ops().wide_attn_bwd(Hb, inst, mask, pk["w1t"], pk["w1"], pk["b1"], pk["w2"], alpha,
                                           de.contiguous().float())
        if ctx.gl is not None and ctx.needs_input_grad[3]:
            glue, p = ctx.gl
            w1p, ns = _wgrad_parts(Hb.reshape(-1, H), dZ, 128)
            glue.add(w1p, glue.map_identity(p["attn_kernel"]), ns)
            X = part.shape[-1]                                            # part [blocks][w2 | b1][X >= H]
            j = np.where(np.arange(X) < H, np.arange(X), -1)
            glue.add(part, glue.map_cat([glue.map_index(p["attn_w2"], j, ("attn_w2", X)),
                                         glue.map_index(p["attn_bias"], j, ("attn_b1", X))]), part.shape[0])
            return dH, None, None, None, None, None, None, None
        dW1 = _wgrad(Hb.reshape(-1, H), dZ, 128) if ctx.needs_input_grad[3] else None
        ps = part.sum(0)
        return dH, None, None, dW1, ps[1, :H], ps[0, :H].unsqueeze(1), None, None


def attention_wide(H, mask, W1, b1, w2):
    """Self-attention pooling (reference model/layer_module.py:49-98) over bf16 BiLSTM outputs
    H [S, L, 2u]: bf16 projection GEMM, tanh / score / masked softmax / pooling in fp32."""
    from ..models import reference as ref
    S, L, D = H.shape
    proj = torch.tanh(ProjBF16.apply(H.reshape(S * L, D), W1).view(S, L, -1) + b1)
    # the score as a broadcast product + row sum, not a [S*L, D] x [D, 1] GEMM: that GEMM's weight
    # gradient (K = S*L = 1.2 M, one output column) ran on ~16 workgroups for 3.6 ms per step
    score = (proj * w2[:, 0]).sum(-1, keepdim=True)                     # [S, L, 1]
    adder = (1.0 - mask.to(score.dtype)).unsqueeze(-1) * ref.MASK_ADDER
    alphas = torch.softmax(score + adder, dim=1)
    # pooling as a broadcast product + sum over time (fp32): as bmm it was a batched GEMV per sentence
    # whose backward GEMVs took ~2.7 ms per step at the paper configuration
    e = (H * alphas).sum(1)
    return e, alphas


def encode_wide(inst, data, p, U: int, keep_prob: float, seed: int, glue=None):
    """Wide GPU encoder: embedding gather + WideBiLSTM + self-attention (GEMM formulation).  ``glue``: the step's
    StepGlue (training, parameters in the flat buffer): the kernel path's gradients go to its scatter-add."""
    from ..models import reference as ref
    if ops().lstm_wide_seq_ok(U):   # hand-written kernels end to end (u in {64, 100, 128})
        wa, p1a, p2a, ma = data
        attn_fused = bool(ops().wide_attn_ok(2 * U, wa.shape[1]))
        packs = None
        if attn_fused:   # every weight pack of the step from ONE gather launch (ops/wide_packs.py)
            from .wide_packs import wide_packs
            D = p["word_embedding"].shape[1] + 2 * p["pos1_embedding"].shape[1]
            packs = wide_packs(p["lstm_fw_kernel"], p["lstm_fw_bias"], p["lstm_bw_kernel"], p["lstm_bw_bias"],
                               p["attn_kernel"], p["attn_bias"], p["attn_w2"], U, D)
        H = WideSeqBiLSTM.apply(inst, wa, p1a, p2a, p["word_embedding"], p["pos1_embedding"], p["pos2_embedding"],
                                p["lstm_fw_kernel"], p["lstm_fw_bias"], p["lstm_bw_kernel"], p["lstm_bw_bias"], U,
                                int(seed), float(keep_prob), bool(getattr(data, "pos_shift", False)), packs,
                                (glue, p) if glue is not None and attn_fused else None)
        if attn_fused:
            mi = ma if ma.dtype == torch.int32 else ma.int()
            return WideAttn.apply(H, inst.int(), mi.contiguous(), p["attn_kernel"], p["attn_bias"], p["attn_w2"],
                                  packs, (glue, p) if glue is not None else None)
        e, alphas = attention_wide(H, ma[inst.long()] > 0, p["attn_kernel"], p["attn_bias"], p["attn_w2"])
        return e, alphas.squeeze(-1)
    word, pos1, pos2, mask = (t[inst.long()] for t in data)
    # the encoder input is built in bf16 (the GEMM operand dtype): half the concat traffic and no
    # separate fp32 -> bf16 pass; autograd casts the fp32 input gradient back for the position tables
    bf = torch.bfloat16
    Xp = torch.cat([SmallTableGather.apply(p["pos1_embedding"], pos1.long()),
                    SmallTableGather.apply(p["pos2_embedding"], pos2.long())], -1)
    X = torch.cat([p["word_embedding"][word.long()].to(bf), Xp.to(bf)], -1)
    H = WideBiLSTM.apply(X, p["lstm_fw_kernel"], p["lstm_fw_bias"], p["lstm_bw_kernel"], p["lstm_bw_bias"], U,
                         int(seed), float(keep_prob))
    e, alphas = attention_wide(H, mask > 0, p["attn_kernel"], p["attn_bias"], p["attn_w2"])
    return e, alphas.squeeze(-1)


class TallSkinnyMM(torch.autograd.Function):
    """y = x w for tall x [T, n] and a skinny weight w [n, m] (m = N classes): the weight gradient
    x^T dy has an [n, m] output that a single GEMM covers with a handful of workgroups over K = T;
    it is computed as 64 K-slices (bmm) and an ordered sum instead (fp32)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w.t() if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            T = x.shape[0]
            nb = 64 if T % 64 == 0 and T >= 4096 else 1
            dw = torch.bmm(x.view(nb, T // nb, -1).transpose(1, 2), dy.contiguous().view(nb, T // nb, -1)).sum(0)
        return dx, dw


def head_wide_ok(H: int, N: int, K: int, R: int, head: str) -> bool:
    """Shapes the hand-written wide head (csrc/kernels/head_wide.hip) covers."""
    o = ops()
    return bool(o.routing_wide_ok(K, H, R)) and bool(o.ntn_wide_epi_ok(N, head == "paper"))


def _split_parts_mm(a: torch.Tensor, b: torch.Tensor, nb: int = 64):
    """(partials [nb, m, n], nb) of a^T b for tall a [T, m], b [T, n] (the slabs _split_sum_mm sums)."""
    T = a.shape[0]
    if T % nb or T < 64 * nb:
        nb = 1
    return torch.bmm(a.view(nb, T // nb, -1).transpose(1, 2), b.view(nb, T // nb, -1)), nb


def _split_sum_mm(a: torch.Tensor, b: torch.Tensor, nb: int = 64) -> torch.Tensor:
    """a^T b (fp32) for tall a [T, m], b [T, n]: K = T split into nb batched slices + an ordered sum."""
    T = a.shape[0]
    if T % nb or T < 64 * nb:
        nb = 1
    return torch.bmm(a.view(nb, T // nb, -1).transpose(1, 2), b.view(nb, T // nb, -1)).sum(0)


def _splitk_nt(a: torch.Tensor, b: torch.Tensor, ns: int) -> torch.Tensor:
    """a b^T in fp32 for a [M, K], b [N, K] with a long K and a small output: K split into ns chunks as ONE
    strided batched GEMM + an ordered sum (deterministic).  The head's dcls = dP M'^T (K = h H = 25,600, a
    [1280, 256] output at the paper configuration) ran as one GEMM on ~44 workgroups: 104 -> 32 us with
    ns = 8 (a round-5 probe, profiles/r5_dcls)."""
    M, K = a.shape
    N = b.shape[0]
    if ns <= 1 or K % ns or not (a.is_cuda and a.is_contiguous() and b.is_contiguous()):
        return torch.mm(a, b.t(), out_dtype=torch.float32)
    c = K // ns
    return torch.bmm(a.view(M, ns, c).transpose(0, 1), b.view(N, ns, c).permute(1, 2, 0),
                     out_dtype=torch.float32).sum(0)


def _wide_head_forward(e, Ws, M, w, b, E, N, K, Q, R, paper):
    """Routing (e_hat GEMM + routing_wide_fwd) -> NTN (P = C M', T = Q P^T as bf16 GEMMs) -> epilogue.
    M' = M permuted to [a, (s, b')] so that P [E*N, h*H] viewed [E, N*h, H] is each episode's
    [(class, slice), feature] operand: T[e] = Q[e] P[e]^T is ONE batched GEMM with columns c*h + s."""
    o = ops()
    H, h = e.shape[1], M.shape[2]
    NK, NQ = N * K, N * Q
    ev = e.view(E, NK + NQ, H)
    sup = ev[:, :NK].reshape(E * NK, H).float()
    eh = torch.mm(sup, Ws.detach().float())                                     # [E*NK, H] fp32
    cls, cls_bf = o.routing_wide_fwd(eh, E * N, K, R)
    Mt = o.transpose12(M.detach().contiguous(), True).view(H, h * H)             # [a, s*H + b'] bf16
    P = torch.mm(cls_bf, Mt)                                                    # [E*N, h*H] bf16
    qb = ev[:, NK:].to(torch.bfloat16).contiguous()                             # [E, NQ, H]
    T = torch.bmm(qb, P.view(E, N * h, H).transpose(1, 2), out_dtype=torch.float32)   # [E, NQ, N*h]
    wf = w.detach().float().contiguous().view(-1)
    probs = o.ntn_wide_epi_fwd(T, N, h, wf, b.detach().float().contiguous().view(-1), paper)
    return probs.view(E, NQ, N), (sup, eh, cls_bf, Mt, P, qb, T, wf)


def _wide_head_backward(ctx, saved, dz, g, gl=None):
    """Shared backward of HeadWideProbsFn / HeadWideLossFn: dz = dL/dlogit [E*NQ, N] (g: upstream scale);
    saved = the forward's (sup, eh, cls_bf, Mt, P, qb, T, wf, Ws).  T is overwritten with ReLU(T) (the FC
    weight-gradient operand): the backward runs once (no retain_graph double backward)."""
    o = ops()
    sup, eh, cls_bf, Mt, P, qb, T, wf, Ws = saved
    E, N, K, Q, R, paper = ctx.cfg
    H, h = sup.shape[1], T.shape[2] // N
    NK, NQ = N * K, N * Q
    dT, dzs = o.ntn_wide_epi_bwd(T, N, h, wf, dz, g, paper)                     # T <- ReLU(T)
    dT = dT.view(E, NQ, N * h)
    dQ = torch.bmm(dT, P.view(E, N * h, H), out_dtype=torch.float32)           # [E, NQ, H]
    dP = torch.bmm(dT.transpose(1, 2), qb)                                      # [E, N*h, H] bf16
    dPf = dP.view(E * N, h * H)
    dcls = _splitk_nt(dPf, Mt, 8)                                              # [E*N, H]
    dMt = torch.mm(cls_bf.t(), dPf, out_dtype=torch.float32)                   # [H, h*H] fp32 (one GEMM: 30 us
    # vs 69 us split 4 + sum at the paper configuration, profiles/r5_dm1 / r5_dws)
    # dM stays on the LDS-tiled transpose (+ autograd's one add): through the glue, the 6.5 M-entry scatter into
    # M's [a][b][s] layout ran as 102,400 single-row finish workgroups, ~100 us at the paper configuration
    dM = o.transpose12(dMt.view(H, h, H), False)                                 # [a][b][s] fp32
    if gl is not None:   # (StepGlue, W_s, M, ntn_w, ntn_b): the other head gradients into the glue's scatter-add
        glue, pWs, pM, pw, pb = gl
    deh = o.routing_wide_bwd(eh, dcls, E * N, K, R)                            # [E*NK, H]
    ns = 4 if sup.is_cuda and sup.shape[0] % 4 == 0 and sup.shape[0] >= 4096 else 1
    # (fp32 split-K 4 + ordered sum: 26 vs 44 us for one GEMM at the paper configuration, profiles/r5_dm1 / r5_dws)
    wsp = (torch.bmm(sup.view(ns, -1, H).transpose(1, 2), deh.view(ns, -1, H)) if ns > 1
           else torch.mm(sup.t(), deh).unsqueeze(0))
    dsup = torch.mm(deh, Ws.t())
    de = torch.cat([dsup.view(E, NK, H), dQ], 1).view(E * (NK + NQ), H)
    V = T.view(E * NQ, N * h)
    if gl is not None:
        glue.add(wsp, glue.map_identity(pWs), ns)
        if paper:
            wp, nb = _split_parts_mm(V.view(-1, h), dzs.view(-1, 1))           # [nb, h, 1] -> ntn_w [h, 1]
            glue.add(wp, glue.map_identity(pw), nb)
            glue.add(dzs.reshape(-1, 1), glue.map_identity(pb), dzs.numel())  # db = sum of dz
        else:
            wp, nb = _split_parts_mm(V, dzs)                                  # [nb, N*h (c*h + s), N]
            c, sh, c2 = np.meshgrid(np.arange(N), np.arange(h), np.arange(N), indexing="ij")
            glue.add(wp, glue.map_index(pw, ((sh * N + c) * N + c2).reshape(-1), ("ntn_w_ref", N, h)), nb)
            glue.add(dzs, glue.map_identity(pb), dzs.shape[0])
        return de, None, dM, None, None
    dWs = wsp.sum(0) if ns > 1 else wsp[0]
    if paper:
        dw = _split_sum_mm(V.view(-1, h), dzs.view(-1, 1))                     # [h, 1]
        db = dzs.sum().view(1)
    else:
        dw = _split_sum_mm(V, dzs).view(N, h, N).permute(1, 0, 2).reshape(h * N, N)   # row s*N + c
        db = dzs.sum(0)
    return de, dWs, dM, dw, db


class HeadWideProbsFn(torch.autograd.Function):
    """Wide routing + NTN head -> probs, differentiable w.r.t. e and the head parameters."""

    @staticmethod
    def forward(ctx, e, Ws, M, w, b, cfg):
        E, N, K, Q, R, paper = cfg
        probs, saved = _wide_head_forward(e, Ws, M, w, b, E, N, K, Q, R, paper)
        # the output is saved through save_for_backward (an attribute would form a ctx <-> output cycle)
        ctx.save_for_backward(*saved, Ws.detach().float(), probs)
        ctx.cfg = cfg
        ctx.edtype = e.dtype
        return probs

    @staticmethod
    def backward(ctx, dprobs):
        saved = ctx.saved_tensors
        p = saved[-1]
        dz = (dprobs * p * (1.0 - p)).float().contiguous().view(-1, ctx.cfg[1])
        g = torch.empty(0, device=dz.device)
        de, dWs, dM, dw, db = _wide_head_backward(ctx, saved[:-1], dz, g)
        return de.to(ctx.edtype), dWs, dM, dw, db, None


class HeadWideLossFn(torch.autograd.Function):
    """Wide routing + NTN + sigmoid + loss (MSE / CE) + accuracy in one autograd node: the loss,
    accuracy and dL/dlogit come from ina.head_loss (glue.hip) in one launch; the backward scales dz by
    the upstream loss gradient on the device.  Returns (loss, accuracy, probs)."""

    LOSS_BLOCKS = 64

    @staticmethod
    def forward(ctx, e, Ws, M, w, b, labels, cfg, loss_type, reduction, glue=None):
        o = ops()
        E, N, K, Q, R, paper = cfg
        probs, saved = _wide_head_forward(e, Ws, M, w, b, E, N, K, Q, R, paper)
        rows = E * N * Q
        ce = loss_type != "mse"
        mode = {"mse": 0, "ce": 1, "ce_nota": 2}[loss_type]
        scale = (1.0 / rows if ce else 1.0 / (rows * N)) if reduction == "mean" else 1.0 / max(1, E)
        dz = torch.empty(rows, N, dtype=torch.float32, device=e.device)
        out = torch.empty(N + 3, dtype=torch.float32, device=e.device)
        blocks = max(1, min(HeadWideLossFn.LOSS_BLOCKS, (rows + 255) // 256))
        part = torch.empty(blocks * 18, dtype=torch.float32, device=e.device)
        o.head_loss(probs.view(rows, N), labels.reshape(-1).int().contiguous(), scale, dz, out, part, blocks, mode)
        ctx.save_for_backward(*saved, Ws.detach().float())
        ctx.dz = dz
        ctx.cfg = cfg
        ctx.edtype = e.dtype
        ctx.gl = (glue, Ws, M, w, b) if glue is not None else None
        ctx.set_materialize_grads(False)
        loss, acc = out[0], out[1]
        ctx.mark_non_differentiable(acc, probs)
        return loss, acc, probs

    @staticmethod
    def backward(ctx, gloss, _gacc, _gprobs):
        g = (gloss.reshape(1).float().contiguous() if gloss is not None
             else torch.zeros(1, device=ctx.dz.device))
        de, dWs, dM, dw, db = _wide_head_backward(ctx, ctx.saved_tensors, ctx.dz, g, ctx.gl)
        return de.to(ctx.edtype), dWs, dM, dw, db, None, None, None, None, None


def head_wide(e, p, B: int, N: int, K: int, Q: int, iters: int, head: str):
    """Routing + relation head at widths outside the fused kernels (the paper's H = 2u = 256): the
    hand-written wide head (head_wide.hip + GEMMs) when it covers the shape, else the GEMM formulation."""
    if head_wide_ok(e.shape[-1], N, K, iters, head):
        return HeadWideProbsFn.apply(e, p["W_s"], p["M"], p["ntn_w"], p["ntn_b"], (B, N, K, Q, iters, head == "paper"))
    return head_wide_torch(e, p, B, N, K, Q, iters, head)


def head_wide_loss(e, p, labels, B: int, N: int, K: int, Q: int, iters: int, head: str, loss_type: str,
                   reduction: str, glue=None):
    """(loss, accuracy, probs) of the wide head with the fused loss kernel (``glue``: gradients into the step
    glue's scatter-add, see WideSeqBiLSTM)."""
    return HeadWideLossFn.apply(e, p["W_s"], p["M"], p["ntn_w"], p["ntn_b"], labels,
                                (B, N, K, Q, iters, head == "paper"), loss_type, reduction, glue)


def head_wide_torch(e, p, B: int, N: int, K: int, Q: int, iters: int, head: str):
    """Routing + relation head at widths outside the fused kernels (the paper's H = 2u = 256):
    dynamic routing in fp32 (models/reference.py), the neural tensor layer's two contractions
    (P = C M over all classes at once, then T = Q P per episode) as bf16 MFMA GEMMs with
    fp32 accumulation -- the precision of the fused bf16 NTN kernel -- and ReLU / FC / sigmoid in fp32."""
    from ..models import reference as ref
    H = e.shape[-1]
    ev = e.float().view(B, N * K + N * Q, H)
    cls = ref.dynamic_routing(ev[:, : N * K].reshape(B, N, K, H), p["W_s"], iters)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        T = ref.ntn_features(cls, ev[:, N * K:], p["M"])              # [B, NQ, h, N]
    V = torch.relu(T.float())
    h = V.shape[2]
    if head == "reference":
        logits = TallSkinnyMM.apply(V.reshape(B * N * Q, h * N), p["ntn_w"]).view(B, N * Q, N) + p["ntn_b"]
    else:
        logits = torch.einsum("bqsn,s->bqn", V, p["ntn_w"][:, 0]) + p["ntn_b"]
    return torch.sigmoid(logits)
