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
