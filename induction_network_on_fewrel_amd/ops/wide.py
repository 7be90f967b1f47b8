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

import torch

from ._ext import ops


def _wgrad(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a^T b in fp32 for tall bf16 a [T, m], b [T, n] (K = T split into 16 chunks)."""
    T = a.shape[0]
    if T % 16 == 0 and T >= 4096:
        part = torch.bmm(a.view(16, T // 16, -1).transpose(1, 2), b.view(16, T // 16, -1), out_dtype=torch.float32)
        return part.sum(0)
    return torch.mm(a.t(), b, out_dtype=torch.float32)


class WideBiLSTM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Kf, bf, Kb, bb, U, seed, keep_prob):
        """X [S, L, D] fp32 (gathered embeddings) -> dropout output [S, L, 2U] bf16."""
        o = ops()
        S, L, D = X.shape
        dev = X.device
        Wx = torch.stack([Kf[:D], Kb[:D]]).detach().to(torch.bfloat16)            # [2, D, 4U]
        Wh = torch.stack([Kf[D:], Kb[D:]]).detach().to(torch.bfloat16)            # [2, U, 4U]
        b = torch.stack([bf, bb]).detach().float()                                # [2, 4U]
        Xb = X.detach().reshape(S * L, D).to(torch.bfloat16)
        gx = torch.stack([torch.mm(Xb, Wx[d], out_dtype=torch.float32) + b[d] for d in range(2)])
        gx = gx.view(2, S, L, 4 * U).contiguous()
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
        dGcur = torch.empty(2, S, 4 * U, device=dev, dtype=torch.bfloat16)
        WhT = Wh.transpose(1, 2).contiguous()                                    # [2, 4U, U]
        for tau in reversed(range(L)):
            o.lstm_wide_bwd_step(dH, dhrec, dcrec, call, acts, dG, dGcur, tau, seed, kp)
            if tau > 0:
                dhrec = torch.bmm(dGcur, WhT, out_dtype=torch.float32)
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
        return dX.view(S, L, D), dKs[0], dbs[0], dKs[1], dbs[1], None, None, None


def encode_wide(inst, data, p, U: int, keep_prob: float, seed: int):
    """Wide GPU encoder: embedding gather + WideBiLSTM + self-attention (GEMM formulation)."""
    from ..models import reference as ref
    word, pos1, pos2, mask = (t[inst.long()] for t in data)
    X = torch.cat([p["word_embedding"][word.long()], p["pos1_embedding"][pos1.long()],
                   p["pos2_embedding"][pos2.long()]], -1).float()
    H = WideBiLSTM.apply(X, p["lstm_fw_kernel"], p["lstm_fw_bias"], p["lstm_bw_kernel"], p["lstm_bw_bias"], U,
                         int(seed), float(keep_prob))
    e, alphas = ref.self_attention(H.float(), mask > 0, p["attn_kernel"], p["attn_bias"], p["attn_w2"])
    return e, alphas.squeeze(-1)
