// Hand-written gfx950 bf16 GEMM family (fp32 accumulation) for the BERT linears and the paper
// configuration's long-K weight gradients (the reference has no BERT: SURVEY 7.2 step 7, BASELINE.json
// config 4; its LSTM gate GEMMs and their autodiff: /root/reference/model/graph.py:34-47):
//
//     NT : C[M, N] = A[M, K] B[N, K]^T     forward  y = x W^T          (A, B K-contiguous rows)
//     NN : C[M, N] = A[M, K] B[K, N]       dgrad    dx = dy W          (B K-major: W [out][in] read as [K][N])
//     TN : C[M, N] = A[K, M]^T B[K, N]     wgrad    dW = dy^T x        (both K-major; K = tokens, split-K)
//
// with the epilogues hipBLASLt has no gfx950 solution for:
//   EPI_PLAIN : out = bf16(C [+ bias])
//   EPI_GELU  : aux = bf16(C + bias) (the pre-activation the backward needs), out = bf16(gelu(C + bias))
//   EPI_DGELU : d = C * gelu'(aux)  ->  out = bf16(d), slab[2 * row_block + wave_row][N] = column sums of d
//               (the FFN-up bias gradient, summed by the step glue in a fixed order)
//   EPI_RES   : out = bf16(C + res) with res = out's previous contents (the residual branch's gradient added by
//               the dgrad GEMM itself: no separate add, no out-of-place copy)
//   EPI_SLAB  : fp32 split-K partial slabs out[split][M][ldo] (summed in a fixed order into the flat gradient:
//               deterministic, no atomics)
//
// Structure: 256x256x64 tiles, 8 waves (2 row groups x 4 column groups), 1 workgroup per CU, all operand
// staging by LDS-DMA (global_load_lds_dwordx4, inline asm: no staging registers, no ds_write) into two
// K-step buffers of four 16-KiB half-tile images (A half 0 / 1, B half 0 / 1).  Each K-step is two phases of
// 32 v_mfma_f32_16x16x32_bf16 between raw s_barriers; the two row groups run one barrier apart (ping-pong:
// on every SIMD one wave issues its MFMA cluster while the other issues its LDS reads and DMA).
//
//   X: read B half 0 / 1 + A half 0 subtiles | stage A1 of step s+1       | MFMA (A0,B0) (A0,B1)
//   Y: read A half 1 subtiles                | stage A0, B0, B1 of s+2    | MFMA (A1,B1) (A1,B0)
// Every phase retires its LDS reads (lgkmcnt(0)) before its barrier, so a half-tile may be restaged one phase
// after its last read (WAR); vmcnt(8) before each phase barrier leaves the 4 most recent half-tiles in flight.
// The waits also serve the row group one barrier BEHIND: its wait before a phase covers every half-tile the
// leading group reads in that phase (e.g. the leading X(s) reads A0 / B0 / B1 of s, which the lagging group's
// Y(s-1) wait retires).  Measured and not kept (profiles/r6_gemm2): 4 + 4 DMAs per phase pair (B1 of s+1 staged
// in X(s): the lagging group's Y wait must then drop to vmcnt(4)) -- equal; no per-cluster s_setprio, or a static
// s_setprio 1 for row group 1 -- 10-35% slower.
//
// Two operand image kinds, same 16 KiB and the same DMA count per thread (2 pieces of 1 KiB per wave):
//   direct (K-contiguous rows [R][ld]): 128 rows x 64 k (128 B); 16-B chunk c of row r at c ^ ((r >> 1) & 7);
//       fragments by ds_read_b128 (16 rows x one chunk per lane group: conflict-free).
//   K-major ([K][ld], the tile's rows are the image's columns): 64 k rows x 128 columns (256 B); 16-B chunk c of
//       row k at c ^ 2 f(k), f(k) = (k & 3) | (k >> 3 & 1) << 2; fragments TRANSPOSED out of the image by two
//       ds_read_b64_tr_b16 (rows 8 q + 0..3 / + 4..7 of a lane group: the 8 rows one 32-lane half reads have
//       distinct f, so its 32 x 8 B are conflict-free).  The tile offset of a read cannot be an immediate (the
//       XOR touches the tile bits), so each lane keeps one address per tile it owns (4 for A, 2 for B).
// LDS-DMA writes lane-linearly, so the swizzles are applied to each lane's SOURCE address.
//
// MFMA operands are swapped (A operand = the B image fragment): the accumulator holds C^T tiles, so a lane
// owns 4 consecutive output columns of one row -> 16-byte stores after two permlane swaps (widen), fp32 slab
// rows as float4, and the bias-gradient column sums are in-lane adds + one 16-lane DPP reduction.
//
// Staging cost (profiles/r6_gpmc): every lane keeps its 8 piece offsets relative to the tile origin; the tile
// origin and the K-step are the uniform soffset, so a K-step's 8 DMAs cost no address VALU.
// Ragged shapes: direct-operand rows past M / N (every thread still issues the same DMA count, so the counted
// waits stay exact) and never stored; K-major operand columns past M / N are
// out of range and never stored (M, N multiples of 8); K-major rows past K are out of range, so a K-major K may be
// any value and split-K ranges may run past it.  Out-of-range pieces are buffer loads at an offset past the
// descriptor's byte count: they write zeros (no clamp, no zero buffer).  Direct operands need K % 64 == 0.
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int G_BM = 256, G_BN = 256, G_BK = 64;
constexpr int G_THREADS = 512;
constexpr int G_HALF = 16384;       // bytes of one half-tile image
constexpr int G_BUF = 4 * G_HALF;   // A0 | A1 | B0 | B1
constexpr int G_LDS = 2 * G_BUF;    // 128 KiB

enum { L_NT = 0, L_NN = 1, L_TN = 2 };

enum { EPI_PLAIN = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_PLAIN_B = 3, EPI_RES = 4, EPI_SLAB = 5 };

struct GemmArgs {
  const unsigned short* A;
  const unsigned short* B;
  const float* bias;
  void* out;                    // bf16 [M][ldo], or fp32 slabs [splits][M][ldo] (EPI_SLAB)
  unsigned short* aux;
  float* slab;                  // EPI_DGELU column sums
  int M, N, K, lda, ldb, ldo, ldx;
  int T;                        // K-steps per split
  int splits;
};

INA_DEVICE u16x8_t lds128(uint32_t a) { return *(const __attribute__((address_space(3))) u16x8_t*)(uintptr_t)a; }
INA_DEVICE s16x4_t ldstr(uint32_t a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(uintptr_t)a);
}
INA_DEVICE u16x8_t cat8(const s16x4_t& lo, const s16x4_t& hi) {
  return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                 (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
}
// 16x16x32 fragment of a K-major image at a lane's tile address (rows 8 q + 0..3 and 8 q + 4..7)
INA_DEVICE u16x8_t frag_tr(uint32_t a) { return cat8(ldstr(a), ldstr(a + 4 * 256)); }
INA_DEVICE void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
INA_DEVICE void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
INA_DEVICE void wait_vm() {
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
INA_DEVICE int kswz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// erf(u / sqrt 2) and exp(-u^2 / 2) (Abramowitz-Stegun 7.1.26, |error| <= 1.5e-7): the Gaussian factor is
// shared by GELU'(u) = (1 + erf) / 2 + u exp(-u^2/2) / sqrt(2 pi)
INA_DEVICE void erf_gauss(float u, float& erfv, float& g) {
  const float x = fabsf(u) * 0.70710678118654752f;
  const float t = fast_rcp(fmaf(0.3275911f, x, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  g = __builtin_amdgcn_exp2f(u * u * -0.72134752044448170f);  // exp(-u^2/2)
  erfv = copysignf(fmaf(-p, g, 1.0f), u);
}
INA_DEVICE float gelu_v(float u) {
  float e, g;
  erf_gauss(u, e, g);
  return 0.5f * u * (1.0f + e);
}
INA_DEVICE float gelu_d(float u) {
  float e, g;
  erf_gauss(u, e, g);
  return fmaf(0.5f, e, 0.5f) + u * g * 0.3989422804014327f;
}

struct Frags {
  u16x8_t a0[4][2], a1[4][2];  // A-half 0 / 1 subtiles [m tile][k32 step]
  u16x8_t b0[2][2], b1[2][2];  // B-half 0 / 1 subtiles [n tile][k32 step]
};

template <int MH, int NH>
INA_DEVICE void mma_quadrant(f32x4_t (&acc)[8][4], const u16x8_t (&fa)[4][2], const u16x8_t (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[MH * 4 + i][NH * 2 + j] = mfma_bf16(fb[j][kk], fa[i][kk], acc[MH * 4 + i][NH * 2 + j]);
  __builtin_amdgcn_s_setprio(0);
}

// XCD-aware bijective tile order: the tiles one XCD runs (ti = its blocks' ids + j * grid, all == xcd mod 8
// because the grid is a multiple of 8 or a single round) get consecutive tile ids, so the operand panels of the
// tiles running at once stay in that XCD's L2 (same split, neighbouring row / column tiles).
struct TilePos {
  int m, n, k;   // row / column origin, first absolute K-step
};
INA_DEVICE TilePos tile_coords(int ti, int NT, int MB, int NB, int T) {
  const int xcd = ti & 7, q8 = NT >> 3, r8 = NT & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (ti >> 3);
  const int per = MB * NB, sp = wgid / per, rem = wgid - sp * per;
  return TilePos{(rem / NB) * G_BM, (rem % NB) * G_BN, sp * T};
}

extern __shared__ __attribute__((aligned(16))) unsigned char gemm_lds[];

// Two 16-byte-per-lane LDS-DMA pieces (1 KiB each, lane-linear from the wave-uniform LDS byte addresses dst / dst +
// 1024) by buffer loads: per-lane voffset, uniform soffset, one M0 save / restore for both (cdna_hip_programming.md
// 5.7: M0 is written in the statement that reads it; s_nop 4 covers an soffset / descriptor fresh from a
// v_readfirstlane, s_nop 0 the M0 write -> LDS-DMA).  A voffset of 0x80000000 is out of range: the piece reads zeros.
INA_DEVICE void bdma2(__amdgpu_buffer_rsrc_t rs, uint32_t v0, uint32_t v1, uint32_t soff, uint32_t dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, %5 offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %5 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(rs), "s"(dst), "s"(soff)
      : "memory");
}
constexpr uint32_t OOB = 0x80000000u;   // > every descriptor's byte count (operands < 2 GiB: checked on the host)

// One operand's DMA geometry.  KMAJ = false: direct image of rows [R][ld] (K contiguous); true: K-major image.
// voff[h][j]: the lane's byte offset of piece j of half h relative to the tile origin (tile-invariant); the tile's
// rows / columns and the K-step go into the uniform soffset.  Rows / columns past the operand (the last tile) and
// K-major rows past K take the out-of-range offset (a uniform branch decides whether any lane needs the check).
template <bool KMAJ>
struct OpStage {
  __amdgpu_buffer_rsrc_t rs;
  int ld2;    // row stride in bytes
  int lim;    // direct: rows R; K-major: columns C
  int K;
  uint32_t voff[2][2];
  INA_DEVICE void init(int w, int lane, const unsigned short* base, int ld, int width, int rows, int Kk) {
    ld2 = ld * 2;
    lim = KMAJ ? width : rows;
    K = Kk;
    // byte count: through the last row's last element (a column slice of wider rows ends before its row stride)
    const uint32_t bytes = (uint32_t)((size_t)(rows - 1) * ld2 + (size_t)width * 2);
    rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(base), (short)0, (int)bytes, 0x00020000);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (!KMAJ) {
          const int r = 16 * w + 8 * j + (lane >> 3);
          voff[h][j] = (uint32_t)((h * 128 + r) * ld2 + ((lane & 7) ^ ((r >> 1) & 7)) * 16);
        } else {
          const int r = 8 * w + 4 * j + (lane >> 4);
          voff[h][j] = (uint32_t)(r * ld2 + (h * 128 + 8 * ((lane & 15) ^ kswz(r))) * 2);
        }
      }
  }
  // half h (0, 1) of the tile whose rows (direct) / columns (K-major) start at row0, absolute K-step kt ->
  // LDS byte address dst (this wave's first piece)
  INA_DEVICE void stage(uint32_t dst, int row0, int h, int kt) const {
    uint32_t v0 = voff[h][0], v1 = voff[h][1];
    uint32_t soff;
    if constexpr (!KMAJ) {
      soff = (uint32_t)(row0 * ld2 + kt * (G_BK * 2));
      if (row0 + 256 > lim) {   // ragged last row tile
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const int r0 = row0 + h * 128 + 16 * w + (lane >> 3);
        v0 = r0 < lim ? v0 : OOB;
        v1 = r0 + 8 < lim ? v1 : OOB;
      }
    } else {
      soff = (uint32_t)(kt * G_BK * ld2 + row0 * 2);
      if (row0 + 256 > lim || (kt + 1) * G_BK > K) {   // ragged last column tile / K tail
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        // pieces 0 / 1: image rows r and r + 4 (same swizzle), the same logical column chunk
        const int r = 8 * w + (lane >> 4), k = kt * G_BK + r;
        const int c = row0 + h * 128 + 8 * ((lane & 15) ^ kswz(r));
        v0 = (c < lim && k < K) ? v0 : OOB;
        v1 = (c < lim && k + 4 < K) ? v1 : OOB;
      }
    }
    bdma2(rs, v0, v1, soff, dst);
  }
};

// LDS byte offsets of this lane's fragment reads inside a half-tile image.  Direct: rd[kk] for tile 0 (tile i at
// + i * 16 rows * 128 B).  K-major: tr[t] for each owned tile t at kk = 0 (kk = 1 at + 32 rows * 256 B).
template <bool KMAJ, int NTILE>
struct OpRead {
  uint32_t o[KMAJ ? NTILE : 2];
  INA_DEVICE void init(int tile0, int lane) {
    const int fr = lane & 15, fq = lane >> 4;
    if constexpr (!KMAJ) {
      o[0] = (uint32_t)((16 * tile0 + fr) * 128 + ((fq ^ (fr >> 1)) * 16));
      o[1] = (uint32_t)((16 * tile0 + fr) * 128 + (((4 + fq) ^ (fr >> 1)) * 16));
    } else {
      const int row = 8 * fq + (fr >> 2), sw = kswz(row);
#pragma unroll
      for (int t = 0; t < NTILE; ++t)
        o[t] = (uint32_t)(row * 256 + (((2 * (tile0 + t) + ((fr >> 1) & 1)) ^ sw) << 4) + (fr & 1) * 8);
    }
  }
  INA_DEVICE u16x8_t frag(uint32_t img, int t, int kk) const {
    if constexpr (!KMAJ) return lds128(img + o[kk] + t * 16 * 128);
    else return frag_tr(img + o[t] + kk * 32 * 256);
  }
};

template <int LAYOUT>
struct Ops {
  static constexpr bool TA = LAYOUT == L_TN, TB = LAYOUT != L_NT;
  OpStage<TA> sa;
  OpStage<TB> sb;
  OpRead<TA, 4> ra;
  OpRead<TB, 2> rb;
  uint32_t dst0;   // this wave's first DMA piece in a half-tile image (wave-uniform: an SGPR for M0)
  INA_DEVICE void stage(int buf, int H, const TilePos& p) const {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(dst0 + buf * G_BUF + H * G_HALF);
    if (H < 2) sa.stage(dst, p.m, H, p.k);
    else sb.stage(dst, p.n, H - 2, p.k);
  }
};

// One K-step (2 phases) on buffer BUF.  full: step s+2 exists (steady-state counted waits); otherwise every wait
// is vmcnt(0).  p1 / p2: the staging positions of steps s+1 / s+2, valid if st1 / st2.
template <int BUF, int LAYOUT>
INA_DEVICE void kstep(f32x4_t (&acc)[8][4], Frags& f, const Ops<LAYOUT>& op, bool full, bool st1, bool st2,
                      const TilePos& p1, const TilePos& p2) {
  constexpr int OTHER = BUF ^ 1;
  const uint32_t buf = lds_addr(gemm_lds) + BUF * G_BUF;
  auto read_a = [&](u16x8_t (&fa)[4][2], int H) {
    const uint32_t img = buf + H * G_HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = op.ra.frag(img, i, 0);
      fa[i][1] = op.ra.frag(img, i, 1);
    }
  };
  auto read_b = [&](u16x8_t (&fb)[2][2], int H) {
    const uint32_t img = buf + (2 + H) * G_HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[j][0] = op.rb.frag(img, j, 0);
      fb[j][1] = op.rb.frag(img, j, 1);
    }
  };
  // X: A0 / B0 / B1 subtiles, quadrants (A0,B0) (A0,B1); stage A1 of s+1; A1 of s must land before Y
  read_b(f.b0, 0);
  read_b(f.b1, 1);
  read_a(f.a0, 0);
  if (st1) op.stage(OTHER, 1, p1);
  wait_lgkm0();
  if (full) wait_vm<8>(); else wait_vm<0>();
  barrier();
  mma_quadrant<0, 0>(acc, f.a0, f.b0);
  mma_quadrant<0, 1>(acc, f.a0, f.b1);
  barrier();
  // Y: A1 subtile, quadrants (A1,B1) (A1,B0); restage A0 / B0 / B1 (read in X) with s+2; A0 / B0 / B1 of s+1
  // must land before its X
  read_a(f.a1, 1);
  if (st2) {
    op.stage(BUF, 0, p2);
    op.stage(BUF, 2, p2);
    op.stage(BUF, 3, p2);
  }
  wait_lgkm0();
  if (full) wait_vm<8>(); else wait_vm<0>();
  barrier();
  mma_quadrant<1, 1>(acc, f.a1, f.b1);
  mma_quadrant<1, 0>(acc, f.a1, f.b0);
  barrier();
}

// acc[mt][nt][r] = C[m0 + mrow(mt) + fr][n0 + ncol(nt) + 4 fq + r]
INA_DEVICE int erow(int m0, int mt, int wr, int fr) { return m0 + (mt >> 2) * 128 + wr * 64 + (mt & 3) * 16 + fr; }
INA_DEVICE int ecol(int n0, int nt, int wc, int fq) { return n0 + (nt >> 1) * 128 + wc * 32 + (nt & 1) * 16 + 4 * fq; }

// EPI_DGELU / EPI_RES: per (row tile mt, half h) ONE 16-byte load per lane of aux / res (the widened layout,
// unwidened in registers), all 16 issued before the first use; the result in the accumulator layout (bias-gradient
// column sums as before), stored widened.
template <int EPI>
INA_DEVICE void epilogue_rowload(const f32x4_t (&acc)[8][4], const GemmArgs& g, int m0, int n0, int wr, int wc,
                                 int fr, int fq) {
  const unsigned short* src = EPI == EPI_DGELU ? g.aux : reinterpret_cast<const unsigned short*>(g.out);
  const int lds = EPI == EPI_DGELU ? g.ldx : g.ldo;
  unsigned short* out = reinterpret_cast<unsigned short*>(g.out);
  uint4 xa[8][2];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = erow(m0, mt, wr, fr);
    const size_t mrow = (size_t)(m < g.M ? m : 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = n0 + h * 128 + wc * 32 + 8 * fq;
      xa[mt][h] = *reinterpret_cast<const uint4*>(src + mrow * lds + (n < g.N ? n : 0));
    }
  }
  float cs[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[nt][r] = 0.f;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = erow(m0, mt, wr, fr);
    const bool ok = m < g.M;
    const size_t mrow = (size_t)(ok ? m : 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint2 ax = uint2{xa[mt][h].x, xa[mt][h].y}, ay = uint2{xa[mt][h].z, xa[mt][h].w};
      unwiden(ax, ay);
      const u16x4_t xv[2] = {__builtin_bit_cast(u16x4_t, ax), __builtin_bit_cast(u16x4_t, ay)};
      u16x4_t o[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool cok = ok && ecol(n0, 2 * h + j, wc, fq) < g.N;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (EPI == EPI_DGELU) {
            const float d = cok ? acc[mt][2 * h + j][r] * gelu_d(bf2f(xv[j][r])) : 0.f;
            o[j][r] = f2bf(d);
            cs[2 * h + j][r] += d;
          } else {
            o[j][r] = f2bf(acc[mt][2 * h + j][r] + bf2f(xv[j][r]));
          }
        }
      }
      uint2 X = __builtin_bit_cast(uint2, o[0]), Y = __builtin_bit_cast(uint2, o[1]);
      widen(X, Y);
      const int n = n0 + h * 128 + wc * 32 + 8 * fq;
      if (ok && n < g.N) *reinterpret_cast<uint4*>(out + mrow * g.ldo + n) = uint4{X.x, X.y, Y.x, Y.y};
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    float* srow = g.slab + (size_t)(2 * (m0 / G_BM) + wr) * g.N;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float4 sv;
      sv.x = group16_sum(cs[nt][0]);
      sv.y = group16_sum(cs[nt][1]);
      sv.z = group16_sum(cs[nt][2]);
      sv.w = group16_sum(cs[nt][3]);
      const int n = ecol(n0, nt, wc, fq);
      if (fr == 0 && n < g.N) *reinterpret_cast<float4*>(srow + n) = sv;
    }
  }
}

template <int EPI>
INA_DEVICE void epilogue(f32x4_t (&acc)[8][4], const GemmArgs& g, const TilePos& tp, int wr, int wc, int fr, int fq) {
  const int m0 = tp.m, n0 = tp.n;
  if constexpr (EPI == EPI_DGELU || EPI == EPI_RES) {
    epilogue_rowload<EPI>(acc, g, m0, n0, wr, wc, fr, fq);
    return;
  }
  if constexpr (EPI == EPI_SLAB) {
    float* out = reinterpret_cast<float*>(g.out) + (size_t)(tp.k / g.T) * g.M * g.ldo;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int m = erow(m0, mt, wr, fr);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int n = ecol(n0, nt, wc, fq);
        if (m < g.M && n < g.N) *reinterpret_cast<f32x4_t*>(out + (size_t)m * g.ldo + n) = acc[mt][nt];
      }
    }
    return;
  }
  f32x4_t bb[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = ecol(n0, nt, wc, fq);
    bb[nt] = ((EPI == EPI_GELU || EPI == EPI_PLAIN_B) && n < g.N) ? *reinterpret_cast<const f32x4_t*>(g.bias + n)
                                                                 : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  // consume the bias loads at once: a load still pending where the K loop resumes would make hipcc drain
  // vmcnt (the in-flight DMAs) at the loop head of every K-step
  if constexpr (EPI == EPI_GELU || EPI == EPI_PLAIN_B)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bb[0]), "+v"(bb[1]), "+v"(bb[2]), "+v"(bb[3])::"memory");
  unsigned short* out = reinterpret_cast<unsigned short*>(g.out);
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = erow(m0, mt, wr, fr);
    const bool ok = m < g.M;
    const size_t mrow = (size_t)(ok ? m : 0);
    u16x4_t ov[4], axv[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      u16x4_t o, ax;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float u = acc[mt][nt][r] + bb[nt][r];
        if constexpr (EPI == EPI_GELU) {
          ax[r] = f2bf(u);
          o[r] = f2bf(gelu_v(u));
        } else {
          o[r] = f2bf(u);
        }
      }
      ov[nt] = o;
      axv[nt] = ax;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = n0 + h * 128 + wc * 32 + 8 * fq;
      uint2 X = __builtin_bit_cast(uint2, ov[2 * h]), Y = __builtin_bit_cast(uint2, ov[2 * h + 1]);
      widen(X, Y);
      if (ok && n < g.N) *reinterpret_cast<uint4*>(out + mrow * g.ldo + n) = uint4{X.x, X.y, Y.x, Y.y};
      if constexpr (EPI == EPI_GELU) {
        uint2 Xa = __builtin_bit_cast(uint2, axv[2 * h]), Ya = __builtin_bit_cast(uint2, axv[2 * h + 1]);
        widen(Xa, Ya);
        if (ok && n < g.N) *reinterpret_cast<uint4*>(g.aux + mrow * g.ldx + n) = uint4{Xa.x, Xa.y, Ya.x, Ya.y};
      }
    }
  }
}

// Persistent: block b runs tiles b, b + grid, b + 2 grid, ... as ONE stream of K-steps (s = local tile * T + kt,
// buffer s & 1), so the DMA of the next tile's first two K-steps is in flight during the current tile's last two
// and its epilogue; there is one pipeline fill per block, not per tile.
template <int LAYOUT, int EPI>
__global__ __launch_bounds__(G_THREADS, 1) void gemm_bf16_kernel(GemmArgs g) {
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int MB = (g.M + G_BM - 1) / G_BM, NB = (g.N + G_BN - 1) / G_BN, NT = MB * NB * g.splits;
  const int G = gridDim.x, b = blockIdx.x;
  const int T = g.T;
  const int ntile = (NT - b + G - 1) / G;
  const int S = ntile * T;

  Ops<LAYOUT> op;
  constexpr bool TA = LAYOUT == L_TN, TB = LAYOUT != L_NT;
  op.sa.init(w, lane, g.A, g.lda, TA ? g.M : g.K, TA ? g.K : g.M, g.K);
  op.sb.init(w, lane, g.B, g.ldb, TB ? g.N : g.K, TB ? g.K : g.N, g.K);
  op.ra.init(4 * wr, lane);
  op.rb.init(2 * wc, lane);
  op.dst0 = __builtin_amdgcn_readfirstlane(lds_addr(gemm_lds) + 2 * w * 1024);
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  Frags f;

  // current tile (compute) and the stream positions one and two steps ahead (staging)
  int jt = 0, kt = 0;
  TilePos cur = tile_coords(b, NT, MB, NB, T);
  TilePos p1 = cur, p2 = cur;
  int j2 = 0, k2 = 0;
  auto adv2 = [&]() {   // p1 <- p2, p2 <- the next K-step of the stream
    p1 = p2;
    ++p2.k;
    if (++k2 == T) {
      k2 = 0;
      ++j2;
      if (j2 < ntile) p2 = tile_coords(b + j2 * G, NT, MB, NB, T);
    }
  };
  // prologue: step 0 (A0 B0 B1 A1) and step 1 (A0 B0 B1; its A1 is staged in step 0's X phase)
  for (int p = 0; p < 2 && p < S; ++p) {
    op.stage(p, 0, p2);
    op.stage(p, 2, p2);
    op.stage(p, 3, p2);
    if (p == 0) op.stage(p, 1, p2);
    adv2();
  }
  if (S > 1) wait_vm<8>(); else wait_vm<0>();   // step 0's A0 B0 B1 (every wave's)
  barrier();
  if (wr == 1) barrier();  // ping-pong: row group 1 runs one barrier behind row group 0

  for (int s = 0; s < S; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ss = s + u;
      if (ss < S) {
        const bool st1 = ss + 1 < S, st2 = ss + 2 < S;
        if (u == 0)
          kstep<0>(acc, f, op, st2, st1, st2, p1, p2);
        else
          kstep<1>(acc, f, op, st2, st1, st2, p1, p2);
        adv2();
        if (++kt == T) {
          epilogue<EPI>(acc, g, cur, wr, wc, fr, fq);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          kt = 0;
          if (++jt < ntile) cur = tile_coords(b + jt * G, NT, MB, NB, T);
        }
      }
    }
  }
  if (wr == 0) barrier();  // balance the barrier counts of the two row groups
}

int cu_count() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n < 8)
      return 0;
    ncu = n & ~7;  // a multiple of 8: every block's tiles stay on its XCD (tile_coords)
  }
  return ncu;
}

template <int LAYOUT, int EPI>
int launch_gemm(const GemmArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_kernel<LAYOUT, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            G_LDS) != hipSuccess)
      return 2;
    attr = true;
  }
  const int ncu = cu_count();
  if (ncu == 0) return 3;
  const long tiles = (long)((a.M + G_BM - 1) / G_BM) * ((a.N + G_BN - 1) / G_BN) * a.splits;
  const long grid = tiles < ncu ? tiles : ncu;  // persistent: one workgroup per CU
  hipLaunchKernelGGL((gemm_bf16_kernel<LAYOUT, EPI>), dim3((unsigned)grid), dim3(G_THREADS), G_LDS, st, a);
  INA_CHECK_LAUNCH();
  return 0;
}

template <int LAYOUT>
int dispatch(const GemmArgs& a, int epi, hipStream_t st) {
  switch (epi) {
    case EPI_PLAIN: return a.bias != nullptr ? launch_gemm<LAYOUT, EPI_PLAIN_B>(a, st) : launch_gemm<LAYOUT, EPI_PLAIN>(a, st);
    case EPI_GELU: return launch_gemm<LAYOUT, EPI_GELU>(a, st);
    case EPI_DGELU: return launch_gemm<LAYOUT, EPI_DGELU>(a, st);
    case EPI_RES: return launch_gemm<LAYOUT, EPI_RES>(a, st);
    default: return 1;
  }
}

}  // namespace

namespace ina {

int gemm_bf16_nt(const void* A, int lda, const void* B, int ldb, int M, int N, int K, const float* bias, void* out,
                 int ldo, void* aux, int ldx, float* slab, int epi, hipStream_t st) {
  return gemm_bf16(L_NT, A, lda, B, ldb, M, N, K, bias, out, ldo, aux, ldx, slab, nullptr, epi, 1, st);
}

int gemm_wgrad_splits(int M, int N, int K) {
  const int ncu = cu_count();
  const long tiles = (long)((M + G_BM - 1) / G_BM) * ((N + G_BN - 1) / G_BN);
  const int ks = (K + G_BK - 1) / G_BK;
  long s = tiles > 0 && ncu > 0 ? ncu / tiles : 1;   // one round of persistent workgroups
  if (s > ks / 4) s = ks / 4;                         // >= 4 K-steps per split (pipeline depth)
  return s > 1 ? (int)s : 1;
}

int gemm_bf16(int layout, const void* A, int lda, const void* B, int ldb, int M, int N, int K, const float* bias,
              void* out, int ldo, void* aux, int ldx, float* slab, const void* zero, int epi, int splits, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0 || layout < L_NT || layout > L_TN) return 1;
  const bool ta = layout == L_TN, tb = layout != L_NT;
  // direct operands: K a multiple of 64 (whole K-steps); K-major operands: 16-byte column chunks, rows past K zero
  if ((!ta || !tb) && K % G_BK != 0) return 1;
  (void)zero;
  // buffer descriptors: each operand's bytes < 2 GiB (the out-of-range offset 0x80000000 must exceed them)
  if ((ta ? (long)(K - 1) * lda + M : (long)(M - 1) * lda + K) * 2 >= (1L << 31)) return 1;
  if ((tb ? (long)(K - 1) * ldb + N : (long)(N - 1) * ldb + K) * 2 >= (1L << 31)) return 1;
  if (ta && M % 8 != 0) return 1;
  if (N % 8 != 0) return 1;
  if (lda % 8 != 0 || ldb % 8 != 0 || ldo % (epi == EPI_SLAB ? 4 : 8) != 0 || ldo < N) return 1;
  if (lda < (ta ? M : K) || ldb < (tb ? N : K)) return 1;
  if (((uintptr_t)A & 15) != 0 || ((uintptr_t)B & 15) != 0 || ((uintptr_t)out & 15) != 0 || ((uintptr_t)aux & 15) != 0)
    return 1;
  if (epi == EPI_SLAB && layout != L_TN) return 1;
  if (epi != EPI_SLAB && splits != 1) return 1;
  if ((epi == EPI_GELU || epi == EPI_DGELU) && (aux == nullptr || ldx % 8 != 0 || ldx < N)) return 1;
  if (epi == EPI_GELU && bias == nullptr) return 1;
  if (epi == EPI_DGELU && slab == nullptr) return 1;
  const int ks = (K + G_BK - 1) / G_BK;
  const int T = (ks + splits - 1) / splits;
  if ((long)(splits - 1) * T >= ks) return 1;   // every split has >= 1 K-step
  GemmArgs a{(const unsigned short*)A, (const unsigned short*)B, bias, out,
             (unsigned short*)aux, slab, M, N, K, lda, ldb, ldo, ldx, T, splits};
  if (layout == L_TN) return epi == EPI_SLAB ? launch_gemm<L_TN, EPI_SLAB>(a, st) : 1;
  if (layout == L_NN) return dispatch<L_NN>(a, epi, st);
  return dispatch<L_NT>(a, epi, st);
}

}  // namespace ina
