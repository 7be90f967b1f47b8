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
    host-to-device copies (and HIP-graph capturable).  The key is id(t): never pass a temporary (a
    freed tensor's id is reused, and the cache would return another index table)."""
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
def ntn_slices_per_tile(N: int) -> int:
    """Slices per NTN tile: the rows (slice, class) of a tile fill one 16-row MFMA operand (csrc/kernels/ntn.hip)."""
    return max(1, min(4, 16 // max(1, N)))


def ntn_tile_geometry(H: int, h: int, N: int):
    """-> (MTH, SG, ntile, tile elements (bf16)).  A tile = SG swizzled M images [16 MTH rows a][64 cols b]
    + the 16x16x16 FC fragments W [(s,c)][c'] and Wt [c'][(s,c)] (256 elements each)."""
    MTH = (H + 15) // 16
    SG = ntn_slices_per_tile(N)
    ntile = (h + SG - 1) // SG
    return MTH, SG, ntile, SG * MTH * 16 * 64 + 512


@lru_cache(maxsize=None)
def _ntn_tile_idx(H: int, h: int, N: int, paper: bool):
    """Index tables of the per-step NTN tile pack (csrc/kernels/ntn.hip), element by element:
      mi  [ntile, TE]: (a * H + b) * h + s into M [H, H, h] (-1: zero)
      wi  [ntile, TE]: index into w ([h N, N] reference head, [h, 1] paper head) (-1: zero)
    M image of slice sl: element (a, b) at sl * RA * 64 + a * 64 + 4 (chunk ^ mask_m(a)) + (b & 3), chunk = b >> 2,
    mask_m(a) = {0,0,4,4,8,8,12,12,10,10,14,14,2,2,6,6}[a & 15] (8-byte chunks XOR-swizzled by row: conflict-free
    row and transposed fragment reads; tools/lds_probe/mimage_search.py).
    W fragment (A[i = (s,c)][k = c'], lane l holds row l & 15, k = 4 (l >> 4) + j) and Wt fragment
    (A[i = c'][k = (s,c)]): row (s_loc, c) = divmod(r, N) of the tile; reference head w[(s N + c)][c'],
    paper head w[s] where c == c'."""
    MTH, SG, NT, TE = ntn_tile_geometry(H, h, N)
    RA = 16 * MTH
    mi = np.full((NT, TE), -1, dtype=np.int64)
    wi = np.full((NT, TE), -1, dtype=np.int64)
    t, sl, a, b = np.meshgrid(np.arange(NT), np.arange(SG), np.arange(RA), np.arange(64), indexing="ij")
    s = t * SG + sl
    mask = (0x6622EEAACC884400 >> (4 * (a & 15))) & 15   # csrc/kernels/ntn.hip mask_m
    phys = (((b >> 2) ^ mask) << 2) | (b & 3)
    pos = sl * RA * 64 + a * 64 + phys
    ok = (s < h) & (a < H) & (b < H)
    mi[t, pos] = np.where(ok, (a * H + b) * h + s, -1)
    l, j = np.meshgrid(np.arange(64), np.arange(4), indexing="ij")
    for which, (row, cp) in enumerate(((l & 15, 4 * (l >> 4) + j), (4 * (l >> 4) + j, l & 15))):
        for tt in range(NT):
            sl_, c = row // N, row % N
            ss = tt * SG + sl_
            ok = (row < SG * N) & (ss < h) & (cp < N)
            if paper:
                ok &= c == cp
                idx = ss
            else:
                idx = (ss * N + c) * N + cp
            wi[tt, SG * RA * 64 + 256 * which + l * 4 + j] = np.where(ok, idx, -1)
    return torch.from_numpy(mi), torch.from_numpy(wi)


def pack_ntn_tiles(M: torch.Tensor, w: torch.Tensor, N: int, paper: bool) -> torch.Tensor:
    """M [H, H, h] and the relation FC weight w -> the NTN tile pack (bf16 [ntile, TE])."""
    H, _, h = M.shape
    mi, wi = _ntn_tile_idx(H, h, N, bool(paper))
    dev = M.device
    nm = M.numel()
    flat = torch.cat([M.detach().float().reshape(-1), w.detach().float().reshape(-1), M.new_zeros(1, dtype=torch.float32)])
    mi, wi = _on(mi, dev), _on(wi, dev)
    idx = torch.where(mi >= 0, mi, torch.where(wi >= 0, wi + nm, torch.full_like(mi, flat.numel() - 1)))
    return flat[idx].to(torch.bfloat16).contiguous()


@lru_cache(maxsize=None)
def _ntn_dw_idx(h: int, N: int, paper: bool):
    """dw slab row of ntn_bwd ([ntile][SG N][N] reference / [ntile][SG] paper) -> index into w (-1: dropped)."""
    SG = ntn_slices_per_tile(N)
    NT = (h + SG - 1) // SG
    if paper:
        s = np.arange(NT * SG)
        return torch.from_numpy(np.where(s < h, s, -1))
    t, r, cp = np.meshgrid(np.arange(NT), np.arange(SG * N), np.arange(N), indexing="ij")
    s = t * SG + r // N
    return torch.from_numpy(np.where(s < h, (s * N + r % N) * N + cp, -1).reshape(-1))


# ------------------------------------------------------------------ wide BiLSTM (lstm_wide.hip persistent kernels)
LOG2E = 1.4426950408889634


def wide_shape(U: int):
    """Persistent wide-BiLSTM geometry (csrc/kernels/lstm_wide.hip WideCfg): UP = units padded to 32,
    NW = UP / 16 waves per workgroup (16 units each), 4 forward M-tiles (16 gate rows = 4 units) and UP / 32
    K-steps per wave, G4 = 4 UP permuted gate columns (column 4u + g), G4 / 32 backward K-steps."""
    UP = (U + 31) // 32 * 32
    return dict(UP=UP, NW=UP // 16, M=4, KS=UP // 32, G4=4 * UP, KS2=4 * UP // 32)


def gate_scales(device=None) -> torch.Tensor:
    """exp2 range factor per gate (i, j, f, o): the kernels evaluate sigmoid / tanh as exp2-based forms
    of pre-scaled arguments (ina_common.h sigmoid_l2 / tanh_l2)."""
    return torch.tensor([LOG2E, 2 * LOG2E, LOG2E, LOG2E], dtype=torch.float32, device=device)


@lru_cache(maxsize=None)
def _wide_idx(U: int):
    """Index tables (into a padded [U+1, 4U+1] matrix whose last row / column are zero) for
    * fwd A fragments [NW][M][KS][64][8]: row R = 4q' + g of M-tile m of wave w = gate g of unit
      u = 16w + 4q' + m (lane group q' owns the 4 CONTIGUOUS units 16w + 4q' .. + 3: one 32-byte gate
      load / store and one 8-byte h write per lane and tile); k = 32 ks + 8 (l >> 4) + j = input unit;
      value W_h[k][g U + u]
    * bwd A fragments [NW][KS2][64][8]: row R -> u_in = 16w + R (so the dh accumulator register r of
      lane group q is unit 16w + 4q + r: the forward's lane ownership);
      k = permuted gate column 4 u_out + g; value W_h[u_in][g U + u_out]
    * permuted gate column c = 4u + g -> TF column g U + u (or the zero column)."""
    s = wide_shape(U)
    UP, NW, M, KS, G4, KS2 = s["UP"], s["NW"], s["M"], s["KS"], s["G4"], s["KS2"]
    ZR, ZC = U, 4 * U
    W = 4 * U + 1
    l = np.arange(64)
    R, kg = l & 15, l >> 4
    j = np.arange(8)
    fwd = np.empty((NW, M, KS, 64, 8), dtype=np.int64)
    for w in range(NW):
        for m in range(M):
            u = 16 * w + 4 * (R >> 2) + m
            g = R & 3
            for ks in range(KS):
                k = 32 * ks + 8 * kg[:, None] + j[None, :]
                row = np.where(k < U, k, ZR)
                col = np.where(u < U, g * U + u, ZC)[:, None]
                fwd[w, m, ks] = row * W + np.where(k < U, col, ZC)
    bwd = np.empty((NW, KS2, 64, 8), dtype=np.int64)
    for w in range(NW):
        u_in = 16 * w + R
        for ks in range(KS2):
            k = 32 * ks + 8 * kg[:, None] + j[None, :]
            u_out, g = k >> 2, k & 3
            row = np.where(u_in < U, u_in, ZR)[:, None]
            col = np.where(u_out < U, g * U + u_out, ZC)
            bwd[w, ks] = row * W + col
    c = np.arange(G4)
    u, g = c >> 2, c & 3
    perm = np.where(u < U, g * U + u, ZC)
    gscale = np.array([LOG2E, 2 * LOG2E, LOG2E, LOG2E], dtype=np.float32)[g]
    keep = u < U   # real (unpadded) permuted columns and their TF columns, for unpack_wide_grads
    return (torch.from_numpy(fwd.reshape(-1)), torch.from_numpy(bwd.reshape(-1)), torch.from_numpy(perm),
            torch.from_numpy(gscale), torch.from_numpy(c[keep]), torch.from_numpy(perm[keep]))


def wide_x_cols(D: int) -> int:
    """Row width of the wide path's encoder input Xb: the D = E + 2PD embedding columns, a ones column
    (index D: the x-projection GEMM's bias row, so dW_x's GEMM yields the bias gradient as row D) and
    zero padding to a multiple of 32 (64-byte rows; a K multiple of 32 moves hipBLASLt's x-projection
    GEMM off its edge-tile kernels: 1.60 -> 1.16 ms at the paper configuration, a round-5 probe, profiles/r5_merged)."""
    return (D + 1 + 31) // 32 * 32


def pack_lstm_wide(Kf: torch.Tensor, bf: torch.Tensor, Kb: torch.Tensor, bb: torch.Tensor, U: int, D: int,
                   scaled: bool = True, cast: bool = True):
    """TF BasicLSTMCell kernels [D + U, 4U] + biases of both directions -> the persistent kernels'
    operands (G4 = 4 UP permuted gate columns 4u + g per direction; both directions side by side,
    column dir * G4 + c, so ONE GEMM covers them):
      wxc  [DP, 2 G4] bf16  x-projection, exp2-pre-scaled, zero rows D .. DP (the ones / pad columns
                            of Xb: the fp32 bias is added in-kernel)
      wxcT [2 G4, DP] bf16  wxc transposed (the own GEMM's K-contiguous B operand)
      wxtc [D, 2 G4]  bf16  the same columns UNscaled (dX = dG wxtc^T)
      wxt  [2, D, G4] bf16  per-direction view of wxtc
      bx   [2, G4]    fp32  bias (+1 on the forget gate), pre-scaled
      apk  [2, NW, M, KS, 64, 8] bf16   forward W_h fragments, pre-scaled
      a2pk [2, NW, KS2, 64, 8]   bf16   backward W_h fragments (true weights)
    scaled=False skips the exp2 pre-scales and the forget bias, cast=False keeps fp32: the pure element
    permutation that ops/wide_packs.py turns into one gather index (+ a per-element affine map)."""
    fwd_i, bwd_i, perm, gsc, _, _ = _wide_idx(U)
    dev = Kf.device
    fwd_i, bwd_i, perm, gsc = (_on(t, dev) for t in (fwd_i, bwd_i, perm, gsc))
    DP = wide_x_cols(D)
    outs = {k: [] for k in ("wx", "bx", "wxt", "apk", "a2pk")}
    bfl = (lambda t: t.to(torch.bfloat16)) if cast else (lambda t: t)
    for K, b in ((Kf, bf), (Kb, bb)):
        K = K.detach().float()
        b = b.detach().float()
        Wx = torch.nn.functional.pad(K[:D], (0, 1))                       # [D, 4U+1]
        wxt = Wx[:, perm]                                                 # [D, G4]
        outs["wxt"].append(wxt)
        outs["wx"].append(torch.nn.functional.pad(wxt * gsc if scaled else wxt, (0, 0, 0, DP - D)))
        bfull = torch.nn.functional.pad(b, (0, 1))
        if scaled:
            fb = torch.zeros_like(bfull)
            fb[2 * U:3 * U] = 1.0                                         # TF forget_bias
            outs["bx"].append(((bfull + fb)[perm] * gsc).contiguous())
        else:
            outs["bx"].append(bfull[perm].contiguous())
        Wh = torch.nn.functional.pad(K[D:D + U], (0, 1, 0, 1)).reshape(-1)  # [U+1, 4U+1] flat
        a = Wh[fwd_i].view(-1, 8)
        # fwd fragment scale: the gate of row R = 4q' + g is g = (l & 15) & 3
        gl = (torch.arange(a.shape[0], device=dev) // 1) % 64 % 16 % 4
        outs["apk"].append(bfl(a * gate_scales(dev)[gl][:, None] if scaled else a))
        outs["a2pk"].append(bfl(Wh[bwd_i]))
    wxtc = bfl(torch.cat(outs["wxt"], 1))
    G4 = wxtc.shape[1] // 2
    wxc = bfl(torch.cat(outs["wx"], 1))
    return {"wxc": wxc, "wxcT": wxc.t().contiguous(), "wxtc": wxtc,
            "wxt": wxtc.view(D, 2, G4).transpose(0, 1),
            "bx": torch.stack(outs["bx"]).contiguous(), "apk": torch.stack(outs["apk"]).contiguous(),
            "a2pk": torch.stack(outs["a2pk"]).contiguous()}


def unpack_wide_grads(dwx: torch.Tensor, dwh: torch.Tensor, db: torch.Tensor, U: int):
    """Permuted-gate-column gradients of one direction ([D, G4], [UP, G4], [G4]) -> TF layout
    kernel [D + U, 4U] and bias [4U]."""
    _, _, _, _, src, dst = _wide_idx(U)   # (lru-cached, immortal: safe keys for the device cache)
    src, dst = _on(src, dwx.device), _on(dst, dwx.device)
    K = torch.zeros(dwx.shape[0] + U, 4 * U, device=dwx.device, dtype=torch.float32)
    K[:dwx.shape[0]].index_copy_(1, dst, dwx.float().index_select(1, src))
    K[dwx.shape[0]:].index_copy_(1, dst, dwh[:U].float().index_select(1, src))
    bias = torch.zeros(4 * U, device=db.device, dtype=torch.float32).index_copy_(0, dst, db.float().index_select(0, src))
    return K, bias


@lru_cache(maxsize=None)
def _merged_wgrad_idx(U: int, D: int, DP: int):
    """Flat indices into the merged weight-gradient GEMM's output dwall [DP + 2 UP, 2 G4] (rows
    [x | h_fw | h_bw], columns dir * G4 + permuted gate column; ops/wide.py::WideSeqBiLSTM.backward) for
    BOTH directions' TF-layout gradients at once: out[d] = [D + U + 1, 4U] = kernel rows (x rows, then
    the direction's own h rows) and the bias as the last row (x's ones column, row D of dwall).  One
    gather instead of unpack_wide_grads' zero-fill + index_select + index_copy per block (12 kernels)."""
    _, _, _, _, src, dst = _wide_idx(U)
    UP, G4 = wide_shape(U)["UP"], wide_shape(U)["G4"]
    col = np.empty(4 * U, dtype=np.int64)
    col[dst.numpy()] = src.numpy()                                   # TF column -> permuted column
    rows = np.concatenate([np.arange(D), np.zeros(U, dtype=np.int64), [D]])
    out = np.empty((2, D + U + 1, 4 * U), dtype=np.int64)
    for d in range(2):
        r = rows.copy()
        r[D:D + U] = DP + d * UP + np.arange(U)
        out[d] = r[:, None] * (2 * G4) + d * G4 + col[None, :]
    return torch.from_numpy(out.reshape(-1))


def unpack_merged_wgrad(dwall: torch.Tensor, U: int, D: int):
    """dwall [DP + 2 UP, 2 G4] -> ([dK_fw, dK_bw] each [D + U, 4U], [db_fw, db_bw] each [4U]), fp32."""
    DP = dwall.shape[0] - dwall.shape[1] // 4
    idx = _on(_merged_wgrad_idx(U, D, DP), dwall.device)
    g = dwall.float().reshape(-1).index_select(0, idx).view(2, D + U + 1, 4 * U)
    return [g[0, :D + U], g[1, :D + U]], [g[0, D + U], g[1, D + U]]


@lru_cache(maxsize=None)
def _attn_wide_idx(H: int):
    """Flat indices into a zero-padded [HP, HP] W1 (HP = H rounded up to 32) for the fused attention
    kernels' MFMA A fragments [HP/16 tiles][HP/32 K-steps][64 lanes][8] (csrc/kernels/attn_wide.hip):
    lane l of tile t, K-step ks, element i covers row 16t + (l & 15) and k = 32ks + 8(l >> 4) + i;
    * w1t: A = W1^T (row = output feature j, k = input feature): W1[k][row]   (Z^T = W1^T H^T)
    * w1:  A = W1   (row = input feature k, k = output feature j): W1[row][k]  (dH^T = W1 dZ^T)"""
    HP = (H + 31) // 32 * 32
    t = np.arange(HP // 16)[:, None, None, None]
    ks = np.arange(HP // 32)[None, :, None, None]
    l = np.arange(64)[None, None, :, None]
    i = np.arange(8)[None, None, None, :]
    row = 16 * t + (l & 15)
    kk = 32 * ks + 8 * (l >> 4) + i
    return HP, torch.from_numpy((kk * HP + row).reshape(-1)), torch.from_numpy((row * HP + kk).reshape(-1))


def pack_attn_wide(W1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, cast: bool = True):
    """Self-attention weights (W1 [H, H], b1 [H], w2 [H, 1]) -> the fused attention kernels' operands:
    w1t / w1 bf16 A fragments (see _attn_wide_idx), b1 / w2 fp32 zero-padded to HP."""
    H = W1.shape[0]
    HP, it, iw = _attn_wide_idx(H)
    dev = W1.device
    Wp = torch.zeros(HP, HP, device=dev, dtype=torch.float32)
    Wp[:H, :H] = W1.detach().float()
    flat = Wp.reshape(-1)
    b1p = torch.zeros(HP, device=dev, dtype=torch.float32)
    b1p[:H] = b1.detach().float().reshape(-1)
    w2p = torch.zeros(HP, device=dev, dtype=torch.float32)
    w2p[:H] = w2.detach().float().reshape(-1)
    bfl = (lambda t: t.to(torch.bfloat16)) if cast else (lambda t: t)
    return {"w1t": bfl(flat[_on(it, dev)]), "w1": bfl(flat[_on(iw, dev)]), "b1": b1p, "w2": w2p}
