"""CPU checks of the MFMA weight-fragment packs against a numpy emulation of the fragment layouts
(v_mfma_f32_16x16x32_bf16: lane l holds A[row l & 15][k 8 (l >> 4) + j] and B[k 8 (l >> 4) + j][col l & 15],
D[row 4 (l >> 4) + r][col l & 15]).  Pins the record-layout attention packs (rec_attn.hip,
ops/packing.py::_attn_rec_idx) without a GPU."""
import numpy as np
import pytest
import torch

from induction_network_on_fewrel_amd.ops.packing import _attn_rec_idx


def _mfma(A, B):
    """A, B: [64 lanes][8] fragments -> D [16 rows][16 cols]."""
    Am = np.zeros((16, 32))
    Bm = np.zeros((32, 16))
    for l in range(64):
        for j in range(8):
            Am[l & 15, 8 * (l >> 4) + j] = A[l, j]
            Bm[8 * (l >> 4) + j, l & 15] = B[l, j]
    return Am @ Bm


def _rfeat(idx, q, U):
    U4 = U // 4
    return (idx // U4) * U + 4 * (idx % U4) + q


def _gather(W1, idx):
    We = np.concatenate([W1.reshape(-1), [0.0]])
    return We[idx.numpy()]


@pytest.mark.parametrize("U", [8, 20, 32])
def test_rec_attn_projection_pack(U):
    """w1r: P^T[j][seq] from B = each lane's own record features (lane-permuted K)."""
    rng = np.random.default_rng(U)
    H2, U4 = 2 * U, U // 4
    NV, MT = 2 * U4, (H2 + 15) // 16
    NKR = (NV + 7) // 8
    W1 = rng.standard_normal((H2, H2))
    H = rng.standard_normal((16, H2))          # 16 sequences (MFMA columns)
    pi, _ = _attn_rec_idx(U)
    A = _gather(W1, pi)                        # [MT][NKR][64][8]
    P = H @ W1                                 # [seq][j]
    for m in range(MT):
        D = np.zeros((16, 16))
        for ks in range(NKR):
            B = np.zeros((64, 8))
            for l in range(64):
                for j in range(8):
                    idx = 8 * ks + j
                    if idx < NV:
                        B[l, j] = H[l & 15, _rfeat(idx, l >> 4, U)]
            D += _mfma(A[m, ks], B)
        for row in range(16):
            jj = 16 * m + row
            if jj < H2:
                np.testing.assert_allclose(D[row], P[:, jj], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("U", [8, 20, 32])
def test_rec_attn_dh_pack(U):
    """w1rt: dH^T = W1 dP^T with B = the dP accumulator rows (K = j in accumulator order); output
    rows land on each lane's own record features."""
    rng = np.random.default_rng(100 + U)
    H2, U4 = 2 * U, U // 4
    NV, MT = 2 * U4, (H2 + 15) // 16
    NJ = 4 * MT
    NKS2, NRT = (NJ + 7) // 8, (NV + 3) // 4
    W1 = rng.standard_normal((H2, H2))
    dP = rng.standard_normal((16, H2))         # [seq][j]
    _, ti = _attn_rec_idx(U)
    A = _gather(W1, ti)                        # [NRT][NKS2][64][8]
    dH = dP @ W1.T                             # [seq][i] = sum_j W1[i][j] dP[seq][j]
    for T in range(NRT):
        D = np.zeros((16, 16))
        for ks in range(NKS2):
            B = np.zeros((64, 8))
            for l in range(64):
                qk = l >> 4
                for j in range(8):
                    idx = 8 * ks + j
                    jj = 16 * (idx >> 2) + 4 * qk + (idx & 3)
                    if idx < NJ and jj < H2:
                        B[l, j] = dP[l & 15, jj]
            D += _mfma(A[T, ks], B)
        # accumulator lane (q, n) holds rows 4 q + r: the lane's feature list index 4 T + r
        for q in range(4):
            for r in range(4):
                fi = 4 * T + r
                if fi < NV:
                    np.testing.assert_allclose(D[4 * q + r], dH[:, _rfeat(fi, q, U)], rtol=1e-10, atol=1e-10)


def test_rec_attn_pack_zero_padding():
    """pack slots past the lane's features / projection rows read the appended zero element."""
    for U in (8, 20, 32):
        pi, ti = _attn_rec_idx(U)
        Z = (2 * U) ** 2
        assert int(pi.max()) <= Z and int(ti.max()) <= Z
        assert torch.all((pi >= 0) & (ti >= 0))


def test_wide_lstm_packs_emulated_mfma():
    """ops/packing.py::pack_lstm_wide against a numpy emulation of v_mfma_f32_16x16x32_bf16's lane
    layout (lane l: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]): the forward fragments give each
    lane group q the 4 (pre-scaled) gates of unit 16w + 4q + m in M-tile m, the backward fragments give
    dh of unit 16w + 4q + r in accumulator register r (the forward's ownership), and the permuted x-projection /
    bias columns c = 4u + g round-trip through unpack_wide_grads."""
    import torch
    from induction_network_on_fewrel_amd.ops.packing import (LOG2E, pack_lstm_wide, unpack_wide_grads,
                                                              wide_shape)
    for U, D in ((100, 310), (128, 60), (64, 15)):
        g = torch.Generator().manual_seed(U)
        Kf, Kb = torch.randn(D + U, 4 * U, generator=g), torch.randn(D + U, 4 * U, generator=g)
        bf_, bb_ = torch.randn(4 * U, generator=g), torch.randn(4 * U, generator=g)
        s = wide_shape(U)
        NW, M, KS, G4, KS2, UP = s["NW"], s["M"], s["KS"], s["G4"], s["KS2"], s["UP"]
        p = pack_lstm_wide(Kf, bf_, Kb, bb_, U, D)
        sc = np.array([LOG2E, 2 * LOG2E, LOG2E, LOG2E])
        for d, (K, b) in enumerate(((Kf, bf_), (Kb, bb_))):
            Wh = K[D:].double().numpy()
            rb = lambda x: torch.tensor(x).float().bfloat16().double().numpy()   # the packs' bf16 rounding
            h = np.zeros(UP)
            h[:U] = np.random.default_rng(1).standard_normal(U)
            A = p["apk"][d].float().double().numpy().reshape(NW, M, KS, 64, 8)
            for w in range(NW):
                for m in range(M):
                    acc = np.zeros(16)
                    for ks in range(KS):
                        for lane in range(64):
                            R, kg = lane & 15, lane >> 4
                            acc[R] += sum(A[w, m, ks, lane, j] * h[32 * ks + 8 * kg + j] for j in range(8))
                    for R in range(16):
                        u, gg = 16 * w + 4 * (R >> 2) + m, R & 3
                        wcol = (K[D:, gg * U + u].float() * torch.tensor(sc[gg], dtype=torch.float32)) if u < U else None
                        want = wcol.bfloat16().double().numpy() @ h[:U] if u < U else 0.0
                        assert abs(acc[R] - want) <= 1e-9 * (1 + abs(want)), (U, d, w, m, R)
            dGn = np.random.default_rng(2).standard_normal((4, U))
            dGp = np.zeros(G4)
            for u in range(U):
                dGp[4 * u:4 * u + 4] = dGn[:, u]
            A2 = p["a2pk"][d].float().double().numpy().reshape(NW, KS2, 64, 8)
            for w in range(NW):
                acc = np.zeros(16)
                for ks in range(KS2):
                    for lane in range(64):
                        R, kg = lane & 15, lane >> 4
                        acc[R] += sum(A2[w, ks, lane, j] * dGp[32 * ks + 8 * kg + j] for j in range(8))
                for q in range(4):
                    for r in range(4):
                        u_in = 16 * w + 4 * q + r
                        want = sum(rb(Wh[u_in, gg * U: gg * U + U]) @ dGn[gg] for gg in range(4)) if u_in < U else 0.0
                        assert abs(acc[4 * q + r] - want) <= 1e-9 * (1 + abs(want)), (U, d, w, q, r)
            # x-projection columns / bias, and the gradient un-permutation
            wxt = p["wxt"][d].float()
            assert torch.equal(p["wxtc"][:, d * G4:(d + 1) * G4], p["wxt"][d])
            assert p["wxc"].shape == (-(-(D + 1) // 32) * 32, 2 * G4) and float(p["wxc"][D:].abs().sum()) == 0.0
            assert torch.equal(p["wxcT"], p["wxc"].t())
            assert torch.allclose(wxt[:, 4 * 3 + 2], K[:D, 2 * U + 3].bfloat16().float())
            assert abs(float(p["bx"][d][4 * 5 + 2]) - (float(b[2 * U + 5]) + 1.0) * LOG2E) < 1e-5
            dK, db = unpack_wide_grads(wxt, torch.nn.functional.pad(K[D:].bfloat16().float()[:, :0], (0, G4)),
                                       torch.zeros(G4), U)
            assert torch.allclose(dK[:D], K[:D].bfloat16().float())


def test_attn_wide_fragments():
    """ops/packing.py::pack_attn_wide: fragment element (tile t, K-step ks, lane l, i) of w1t is
    W1[32ks + 8(l>>4) + i][16t + (l&15)] (A = W1^T), of w1 W1[16t + (l&15)][32ks + 8(l>>4) + i] (A = W1);
    zero outside H (H = 200 pads to 224)."""
    import torch
    from induction_network_on_fewrel_amd.ops.packing import pack_attn_wide
    for H in (128, 200, 256):
        HP = (H + 31) // 32 * 32
        W1 = torch.randn(H, H)
        pk = pack_attn_wide(W1, torch.randn(H), torch.randn(H, 1))
        Wp = torch.zeros(HP, HP)
        Wp[:H, :H] = W1.bfloat16().float()
        a = pk["w1t"].float().reshape(HP // 16, HP // 32, 64, 8)
        b = pk["w1"].float().reshape(HP // 16, HP // 32, 64, 8)
        for t, ks, l, i in ((0, 0, 0, 0), (HP // 16 - 1, HP // 32 - 1, 63, 7), (3, 1, 37, 5), (HP // 16 - 2, 2, 22, 3)):
            k, r = 32 * ks + 8 * (l >> 4) + i, 16 * t + (l & 15)
            assert float(a[t, ks, l, i]) == float(Wp[k, r])
            assert float(b[t, ks, l, i]) == float(Wp[r, k])
        assert pk["b1"].shape == (HP,) and float(pk["w2"][H:].abs().sum()) == 0.0


def test_narrow_and_wide_attention_index_helpers_coexist():
    """The fused narrow path's pack index (ops/glue.py -> packing._attn_idx(H2, bf16)) and the wide
    attention's fragments (packing._attn_wide_idx(H)) are separate helpers: a name clash once broke
    every narrow-path step."""
    from induction_network_on_fewrel_amd.ops import packing
    pi, ti = packing._attn_idx(40, True)
    assert pi.numel() > 0 and ti.numel() > 0
    HP, it, iw = packing._attn_wide_idx(256)
    assert HP == 256 and it.numel() == iw.numel() == 256 * 256


@pytest.mark.parametrize("H,h,N,paper", [(40, 100, 5, False), (40, 7, 5, True), (64, 9, 10, False), (16, 5, 3, True),
                                         (40, 1, 4, False)])
def test_ntn_tile_pack_layout(H, h, N, paper):
    """The NTN tile pack (csrc/kernels/ntn.hip) read back through the kernel's addressing: M images
    with the 8-byte-chunk XOR swizzle and the two 16x16x16 FC fragments of every tile."""
    from induction_network_on_fewrel_amd.ops.packing import ntn_tile_geometry, pack_ntn_tiles, _ntn_dw_idx
    g = torch.Generator().manual_seed(0)
    M = torch.randn(H, H, h, generator=g)
    w = torch.randn(h, 1, generator=g) if paper else torch.randn(h * N, N, generator=g)
    pk = pack_ntn_tiles(M, w, N, paper).float()
    MTH, SG, NT, TE = ntn_tile_geometry(H, h, N)
    assert pk.shape == (NT, TE) and (TE * 2) % 1024 == 0
    RA = 16 * MTH
    Mb = M.to(torch.bfloat16).float()
    wb = w.to(torch.bfloat16).float().reshape(-1)
    for t in range(NT):
        for sl in range(SG):
            s = t * SG + sl
            for a in range(RA):
                mask = (0x6622EEAACC884400 >> (4 * (a & 15))) & 15
                for b in range(64):
                    v = pk[t, sl * RA * 64 + a * 64 + ((((b >> 2) ^ mask) << 2) | (b & 3))]
                    ref = Mb[a, b, s] if (s < h and a < H and b < H) else 0.0
                    assert v == ref, (t, sl, a, b)
        base = SG * RA * 64
        for l in range(64):
            for j in range(4):
                for which, (row, cp) in enumerate(((l & 15, 4 * (l >> 4) + j), (4 * (l >> 4) + j, l & 15))):
                    sl, c = divmod(row, N)
                    s = t * SG + sl
                    if row >= SG * N or s >= h or cp >= N:
                        ref = 0.0
                    elif paper:
                        ref = wb[s] if c == cp else 0.0
                    else:
                        ref = wb[(s * N + c) * N + cp]
                    assert pk[t, base + 256 * which + 4 * l + j] == ref
    di = _ntn_dw_idx(h, N, paper)
    assert di.numel() == NT * (SG if paper else SG * N * N)
    valid = di[di >= 0]
    assert valid.unique().numel() == valid.numel() == (h if paper else h * N * N)


def test_unpack_merged_wgrad_matches_per_block_unpack():
    """ops/packing.py::unpack_merged_wgrad (one gather over the merged [x | h_fw | h_bw] x [fw | bw]
    weight-gradient GEMM output) equals unpack_wide_grads applied to each direction's diagonal blocks
    (x rows, the direction's own h rows, bias = row D); the cross-direction blocks are ignored."""
    import torch
    from induction_network_on_fewrel_amd.ops.packing import (unpack_merged_wgrad, unpack_wide_grads, wide_shape,
                                                              wide_x_cols)
    for U, D in ((100, 310), (128, 60), (64, 15)):
        s = wide_shape(U)
        G4, UP = s["G4"], s["UP"]
        DP = wide_x_cols(D)
        dwall = torch.randn(DP + 2 * UP, 2 * G4, generator=torch.Generator().manual_seed(U))
        dKs, dbs = unpack_merged_wgrad(dwall, U, D)
        for d in range(2):
            c = slice(d * G4, (d + 1) * G4)
            dK, db = unpack_wide_grads(dwall[:D, c], dwall[DP + d * UP:DP + (d + 1) * UP, c], dwall[D, c], U)
            assert dKs[d].shape == (D + U, 4 * U) and torch.equal(dKs[d], dK), (U, d)
            assert torch.equal(dbs[d], db), (U, d)
