"""Weight -> MFMA-fragment packing for the gfx950 kernels.

Every kernel consumes its weights as per-lane fragments (``[..][64 lanes][KPL]``, KPL = 8 bf16 for
``v_mfma_f32_16x16x32_bf16`` or 1 f32 for ``v_mfma_f32_16x16x4_f32``) so that each lane issues ONE
16-byte load per fragment. The lane maps mirror the comments in ``csrc/kernels/*.hip``; the index
tables are built once per shape on the host and applied as a single device gather per step.
"""
from __future__ import annotations

from functools import lru_cache

_DEV_CACHE = {}


def _on(t: torch.Tensor, dev) -> torch.Tensor:
    """Device copy of a cached (lru_cache'd, hence immortal) host index tensor, made once: no per-step
    host-to-device copies (and HIP-graph capturable)."""
    key = (id(t), str(dev))
    v = _DEV_CACHE.get(key)
    if v is None:
        v = t.to(dev)
        _DEV_CACHE[key] = v
    return v

import numpy as np
import torch


def _kpl(bf16: bool) -> int:
    return 8 if bf16 else 1


# ------------------------------------------------------------------ LSTM
def lstm_shape(U: int, DIN: int, bf16: bool):
    U4 = U // 4
    NX = 4 if DIN <= 16 else 16
    KPL = _kpl(bf16)
    NSLOT = U4 + NX
    NKS = (NSLOT + KPL - 1) // KPL
    NMT2 = (NSLOT + 3) // 4
    NKS2 = (4 * U4 + KPL - 1) // KPL
    return dict(U4=U4, NX=NX, KPL=KPL, NSLOT=NSLOT, NKS=NKS, NMT=U4, NMT2=NMT2, NKS2=NKS2)


@lru_cache(maxsize=None)
def _lstm_idx(U: int, DIN: int, bf16: bool):
    """Flat indices into W_ext = pad(W [DIN+U, 4U]) -> [DIN+U+1, 4U+1]; zero row/col at the end."""
    s = lstm_shape(U, DIN, bf16)
    U4, NX, KPL, NKS, NMT2, NKS2 = s["U4"], s["NX"], s["KPL"], s["NKS"], s["NMT2"], s["NKS2"]
    ZR, ZC = DIN + U, 4 * U
    W = 4 * U + 1

    def feat(idx, q):
        if idx < U4:
            return DIN + 4 * idx + q
        xi = idx - U4
        f = 4 * xi + q
        return f if (xi < NX and f < DIN) else ZR

    fwd = np.empty((U4, NKS, 64, KPL), dtype=np.int64)
    for m in range(U4):
        for ks in range(NKS):
            for l in range(64):
                q, r = l >> 4, l & 15
                gate = (r & 3) * U + 4 * m + (r >> 2)
                for j in range(KPL):
                    f = feat(ks * KPL + j, q)
                    fwd[m, ks, l, j] = f * W + (gate if f != ZR else ZC)
    bwd = np.empty((NMT2, NKS2, 64, KPL), dtype=np.int64)
    for mt in range(NMT2):
        for ks in range(NKS2):
            for l in range(64):
                r, qk = l & 15, l >> 4
                qr, reg = r >> 2, r & 3
                fs = 4 * mt + reg
                f = feat(fs, qr) if fs < U4 + NX else ZR
                for j in range(KPL):
                    idx = ks * KPL + j
                    gate = (idx & 3) * U + 4 * (idx >> 2) + qk if idx < 4 * U4 else ZC
                    bwd[mt, ks, l, j] = f * W + gate
    return torch.from_numpy(fwd), torch.from_numpy(bwd)


def _pad_lstm(W: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.pad(W, (0, 1, 0, 1))


def pack_lstm(Wf: torch.Tensor, Wb: torch.Tensor, U: int, DIN: int, bf16: bool):
    """-> (apack [2, NMT, NKS, 64, KPL], a2pack [2, NMT2, NKS2, 64, KPL]) in bf16 or fp32."""
    fi, bi = _lstm_idx(U, DIN, bf16)
    dev = Wf.device
    fi, bi = _on(fi, dev), _on(bi, dev)
    dt = torch.bfloat16 if bf16 else torch.float32
    outs_f, outs_b = [], []
    for W in (Wf, Wb):
        We = _pad_lstm(W.detach().float()).reshape(-1)
        outs_f.append(We[fi])
        outs_b.append(We[bi])
    return torch.stack(outs_f).to(dt).contiguous(), torch.stack(outs_b).to(dt).contiguous()


# ------------------------------------------------------------------ attention
@lru_cache(maxsize=None)
def _attn_idx(H2: int, bf16: bool):
    KPL = _kpl(bf16)
    KP = ((H2 + 31) // 32) * 32 if bf16 else ((H2 + 3) // 4) * 4
    NKS = KP // 32 if bf16 else KP // 4
    MT = (H2 + 15) // 16
    NKS2 = (4 * MT + KPL - 1) // KPL
    Z = H2 * H2  # zero element index

    def feat_of(v, q):
        return (v >> 3) * 32 + 8 * q + (v & 7) if bf16 else 4 * v + q

    p = np.empty((MT, NKS, 64, KPL), dtype=np.int64)
    for m in range(MT):
        for ks in range(NKS):
            for l in range(64):
                jo = 16 * m + (l & 15)
                for j in range(KPL):
                    i = feat_of(ks * KPL + j, l >> 4)
                    p[m, ks, l, j] = i * H2 + jo if (i < H2 and jo < H2) else Z
    t = np.empty((MT, NKS2, 64, KPL), dtype=np.int64)
    for m in range(MT):
        for ks in range(NKS2):
            for l in range(64):
                i = 16 * m + (l & 15)
                q = l >> 4
                for j in range(KPL):
                    idx = ks * KPL + j
                    ji = 16 * (idx >> 2) + 4 * q + (idx & 3)
                    t[m, ks, l, j] = i * H2 + ji if (idx < 4 * MT and i < H2 and ji < H2) else Z
    return torch.from_numpy(p), torch.from_numpy(t)


def pack_attn(W1: torch.Tensor, bf16: bool):
    H2 = W1.shape[0]
    pi, ti = _attn_idx(H2, bf16)
    dev = W1.device
    We = torch.cat([W1.detach().float().reshape(-1), W1.new_zeros(1, dtype=torch.float32)])
    dt = torch.bfloat16 if bf16 else torch.float32
    return We[_on(pi, dev)].to(dt).contiguous(), We[_on(ti, dev)].to(dt).contiguous()


@lru_cache(maxsize=None)
def _attn_rec_idx(U: int):
    """Flat indices into [W1 [2U, 2U] | 0] for the record-layout attention kernels (rec_attn.hip).
    Lane group q owns the features rfeat(idx, q) = (idx // U4) * U + 4 * (idx % U4) + q, idx < 2 * U4.
      w1r  [MT][NKR][64][8]:  A[row j = 16 m + (l & 15)][k slot (l >> 4, jj)] = W1[rfeat(8 ks + jj, l >> 4)][j]
      w1rt [NRT][NKS2][64][8]: A[row (qr, rr) = l & 15][k slot (l >> 4, jj)] = W1[rfeat(4 T + rr, qr)][j] with
                              j = 16 (idx >> 2) + 4 (l >> 4) + (idx & 3), idx = 8 ks + jj (dP accumulator order)."""
    U4, H2 = U // 4, 2 * U
    NV, MT = 2 * U4, (H2 + 15) // 16
    NKR, NJ = (NV + 7) // 8, 4 * MT
    NKS2, NRT = (NJ + 7) // 8, (NV + 3) // 4
    Z = H2 * H2

    def rfeat(idx, q):
        return (idx // U4) * U + 4 * (idx % U4) + q

    p = np.full((MT, NKR, 64, 8), Z, dtype=np.int64)
    for m in range(MT):
        for ks in range(NKR):
            for l in range(64):
                j = 16 * m + (l & 15)
                for jj in range(8):
                    idx = 8 * ks + jj
                    if idx < NV and j < H2:
                        p[m, ks, l, jj] = rfeat(idx, l >> 4) * H2 + j
    t = np.full((NRT, NKS2, 64, 8), Z, dtype=np.int64)
    for T in range(NRT):
        for ks in range(NKS2):
            for l in range(64):
                r16 = l & 15
                fi = 4 * T + (r16 & 3)
                if fi >= NV:
                    continue
                i = rfeat(fi, r16 >> 2)
                for jj in range(8):
                    idx = 8 * ks + jj
                    j = 16 * (idx >> 2) + 4 * (l >> 4) + (idx & 3)
                    if idx < NJ and j < H2:
                        t[T, ks, l, jj] = i * H2 + j
    return torch.from_numpy(p), torch.from_numpy(t)


def pack_attn_rec(W1: torch.Tensor):
    """-> (w1r, w1rt) bf16 packs of the record-layout attention kernels (see _attn_rec_idx)."""
    U = W1.shape[0] // 2
    pi, ti = _attn_rec_idx(U)
    dev = W1.device
    We = torch.cat([W1.detach().float().reshape(-1), W1.new_zeros(1, dtype=torch.float32)])
    return We[_on(pi, dev)].to(torch.bfloat16).contiguous(), We[_on(ti, dev)].to(torch.bfloat16).contiguous()


# ------------------------------------------------------------------ NTN (bf16 only)
def _kmap32(q: int, j: int) -> int:
    return 16 * (j >> 2) + 4 * q + (j & 3)


@lru_cache(maxsize=None)
def _ntn_m_idx(H: int, h: int):
    """Packed M fragments for h_pad = 2*ceil(h/2) slices (the pad slice is zero): the NTN kernels
    stage whole slice pairs with global_load_lds and need no per-lane bounds checks."""
    MTH = (H + 15) // 16
    NKA = (MTH + 1) // 2
    Z = H * H * h
    hp = 2 * ((h + 1) // 2)
    mp = np.full((hp, MTH, NKA, 64, 8), Z, dtype=np.int64)
    m2 = np.full((hp, MTH, NKA, 64, 8), Z, dtype=np.int64)
    ls = np.arange(64)
    js = np.arange(8)
    for s in range(h):
        for mb in range(MTH):
            for ka in range(NKA):
                a = 32 * ka + 8 * (ls[:, None] >> 4) + js[None, :]
                b = 16 * mb + (ls[:, None] & 15) + 0 * js[None, :]
                ok = (a < H) & (b < H)
                mp[s, mb, ka] = np.where(ok, (a * H + b) * h + s, Z)
                a2 = 16 * mb + (ls[:, None] & 15) + 0 * js[None, :]
                b2 = 32 * ka + 16 * (js[None, :] >> 2) + 4 * (ls[:, None] >> 4) + (js[None, :] & 3)
                ok2 = (a2 < H) & (b2 < H)
                m2[s, mb, ka] = np.where(ok2, (a2 * H + b2) * h + s, Z)
    return torch.from_numpy(mp), torch.from_numpy(m2)


@lru_cache(maxsize=None)
def _ntn_w_idx(h: int, N: int):
    Z = h * N * N
    npair = (h + 1) // 2
    wp = np.empty((npair, 64, 8), dtype=np.int64)
    wt = np.full((2 * npair, 64, 8), Z, dtype=np.int64)
    for p in range(npair):
        for l in range(64):
            for j in range(8):
                s = 2 * p + (j >> 2)
                c = 4 * (l >> 4) + (j & 3)
                cp = l & 15
                wp[p, l, j] = (s * N + c) * N + cp if (s < h and c < N and cp < N) else Z
    for s in range(h):
        for l in range(64):
            for j in range(8):
                c = l & 15
                cp = 8 * (l >> 4) + j
                wt[s, l, j] = (s * N + c) * N + cp if (c < N and cp < N) else Z
    return torch.from_numpy(wp), torch.from_numpy(wt)


def pack_ntn_M(M: torch.Tensor):
    H, _, h = M.shape
    mi, m2i = _ntn_m_idx(H, h)
    dev = M.device
    Me = torch.cat([M.detach().float().reshape(-1), M.new_zeros(1, dtype=torch.float32)])
    return Me[_on(mi, dev)].to(torch.bfloat16).contiguous(), Me[_on(m2i, dev)].to(torch.bfloat16).contiguous()


def pack_ntn_w(w: torch.Tensor, h: int, N: int):
    wi, wti = _ntn_w_idx(h, N)
    dev = w.device
    we = torch.cat([w.detach().float().reshape(-1), w.new_zeros(1, dtype=torch.float32)])
    return we[_on(wi, dev)].to(torch.bfloat16).contiguous(), we[_on(wti, dev)].to(torch.bfloat16).contiguous()
