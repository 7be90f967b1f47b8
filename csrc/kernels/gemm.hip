// Hand-written gfx950 bf16 GEMM for the BERT feed-forward block (verdict r3 #4; the reference has no
// BERT: SURVEY 7.2 step 7, BASELINE.json config 4):
//
//     C[M, N] = A[M, K] B[N, K]^T      (A and B K-contiguous bf16, fp32 accumulation)
//
// with the epilogues hipBLASLt has no gfx950 solution for:
//   EPI_PLAIN : out = bf16(C + bias)                        (bias optional)
//   EPI_GELU  : aux = bf16(C + bias) (the pre-activation the backward needs), out = bf16(gelu(C + bias))
//   EPI_DGELU : d = C * gelu'(aux)  ->  out = bf16(d), slab[2 * row_block + wave_row][N] = column sums of d
//               (the FFN-up bias gradient, summed by the step glue in a fixed order)
//
// Structure: 256x256x64 tiles, 8 waves (2 row groups x 4 column groups), 1 workgroup per CU, all operand
// staging by LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write) into two K-tile buffers of
// four 16-KiB half-tiles (A rows 0-127 / 128-255, B rows 0-127 / 128-255).  Each K-tile is four phases; a
// phase reads one register subtile (ds_read_b128), issues ONE half-tile of prefetch, and runs 16
// v_mfma_f32_16x16x32_bf16 between two raw s_barriers.  The two row groups run one barrier apart
// (ping-pong): on every SIMD one wave issues its MFMA cluster while the other issues its LDS reads and
// DMA, so the matrix core never waits for an operand.
//
// Phase schedule of K-tile t (buffer t & 1); wave (wr, wc) owns rows {h*128 + wr*64 + [0,64)} and columns
// {h*128 + wc*32 + [0,32)} for h = 0, 1, so every wave reads every half-tile:
//   p0: read A-half 0 + B-half 0 subtiles | stage A1 of tile t+1 | MFMA quadrant (A0, B0)
//   p1: read B-half 1                     | stage A0 of tile t+2 | MFMA (A0, B1)
//   p2: read A-half 1                     | stage B0 of tile t+2 | MFMA (A1, B1)
//   p3: --                                | stage B1 of tile t+2 | vmcnt(6): tile t+1 landed | MFMA (A1, B0)
// Every phase retires its LDS reads (lgkmcnt(0)) before its first barrier, so a half-tile may be restaged
// one phase after its last read (WAR); a DMA'd half-tile is read only in a phase after the counted vmcnt +
// barrier that retires it (RAW).  vmcnt(6) leaves the three most recent half-tiles (6 DMAs per thread) in
// flight across the barrier: a half-tile has 3-6 phases to land.
//
// LDS images are XOR-swizzled (16-B chunk c of image row r stored at chunk c ^ ((r >> 1) & 7)): the
// ds_read_b128 fragment reads (16 rows x one 16-B chunk per lane group) are conflict-free.  Because an
// LDS-DMA writes lane-linearly, the swizzle is applied to the SOURCE address of each lane.
//
// MFMA operands are swapped (A operand = the B image fragment): the accumulator holds C^T tiles, so a lane
// owns 4 consecutive output columns of one row -> 8-byte stores, 8-byte aux loads, and the bias-gradient
// column sums are in-lane adds + one 16-lane DPP reduction.
//
// Ragged M: A rows >= M are clamped to row M - 1 on load (every thread issues the same DMA count, so the
// counted waits stay exact); their outputs are not stored and their d is excluded from the column sums.
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int G_BM = 256, G_BN = 256, G_BK = 64;
constexpr int G_THREADS = 512;
constexpr int G_HALF = 128 * G_BK * 2;  // bytes of one half-tile image (128 rows x 128 B)
constexpr int G_BUF = 4 * G_HALF;       // A0 | A1 | B0 | B1
constexpr int G_LDS = 2 * G_BUF;        // 128 KiB

enum { EPI_PLAIN = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_PLAIN_B = 3 };  // 3: plain + bias (host: epi 0 with a bias)

#ifndef INA_GEMM_STAGGER
#define INA_GEMM_STAGGER 1  // ping-pong the two row groups one barrier apart (0: lockstep, A/B only)
#endif
#ifndef INA_GEMM_LGKM_AFTER
#define INA_GEMM_LGKM_AFTER 0  // 1: retire the phase's LDS reads after its first barrier (A/B only: needs
                               // the 2-phase WAR distance, which the staging schedule does not give)
#endif
#ifndef INA_GEMM_SCHED
#define INA_GEMM_SCHED 2  // operand staging schedule (kstep): 2 two phases per K-step (default: 4-8% over 1),
                          // 1 balanced four phases, 0 front-loaded four phases
#endif
#ifndef INA_GEMM_DIAG
#define INA_GEMM_DIAG 0  // 1: no operand staging inside the K loop (diagnostic of the MFMA/LDS/barrier skeleton)
#endif
#ifndef INA_GEMM_NOSTORE
#define INA_GEMM_NOSTORE 0  // 1: the epilogue stores nothing (diagnostic: the K loop + staging without the C writes)
#endif

struct GemmArgs {
  const unsigned short* A;
  const unsigned short* B;
  const float* bias;
  unsigned short* out;
  unsigned short* aux;
  float* slab;
  int M, N, K, lda, ldb, ldo, ldx;
};

INA_DEVICE void glds16(const unsigned char* gsrc_lane, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc_lane,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
INA_DEVICE u16x8_t ldsr(const unsigned char* p) { return *reinterpret_cast<const u16x8_t*>(p); }
INA_DEVICE void wait_lgkm0() {
  if (!INA_GEMM_LGKM_AFTER) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
INA_DEVICE void barrier() { __builtin_amdgcn_s_barrier(); }

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
// because the grid is a multiple of 8 or a single round) get consecutive tile ids, so the A row panels of
// the tiles running at once stay in that XCD's L2 across the N tiles.
INA_DEVICE void tile_coords(int ti, int NT, int NB, int& m0, int& n0) {
  const int xcd = ti & 7, q8 = NT >> 3, r8 = NT & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (ti >> 3);
  m0 = (wgid / NB) * G_BM;
  n0 = (wgid % NB) * G_BN;
}

// Per-thread DMA geometry: wave w fills image rows 16w .. 16w+15 of every half-tile; piece j (0, 1) covers
// rows 16w + 8j + (lane >> 3), lane's stored chunk lane & 7 <- logical chunk (lane & 7) ^ ((row >> 1) & 7).
// ONE LDS object for everything (a second __shared__ object beside the DMA staging can make hipcc drain
// vmcnt before every LDS read); referenced by symbol so the alias analysis sees the read / DMA offsets.
extern __shared__ __attribute__((aligned(16))) unsigned char gemm_lds[];

struct Stager {
  const unsigned char* gA;
  const unsigned char* gB;
  int lda2, ldb2, M1;       // row strides in bytes, M - 1
  int row[2], chunk[2];     // image row and source byte offset of the chunk, per piece
  int dst0;                 // this wave's first piece in a half-tile image
  // half-tile H (0 A0, 1 A1, 2 B0, 3 B1) of K-step kt of the tile at (m0, n0) into buffer b
  INA_DEVICE void stage(int b, int H, int m0, int n0, int kt) const {
    if (INA_GEMM_DIAG) return;
    unsigned char* dst = gemm_lds + b * G_BUF + H * G_HALF + dst0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned char* src;
      if (H < 2) {
        const int m = min(m0 + H * 128 + row[j], M1);
        src = gA + (size_t)m * lda2 + kt * (G_BK * 2) + chunk[j];
      } else {
        src = gB + (size_t)(n0 + (H - 2) * 128 + row[j]) * ldb2 + kt * (G_BK * 2) + chunk[j];
      }
      glds16(src, dst + j * 1024);
    }
  }
};

template <int N>
INA_DEVICE void wait_vm() {
  if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Staging position of a later K-step of this block's stream: its tile's (m0, n0) and K-step.
struct StagePos {
  int m, n, k;
};

// One K-step (4 phases) on buffer BUF.  full: step s+2 exists (steady-state counted waits); otherwise every
// wait is vmcnt(0).  p1 / p2: the staging positions of steps s+1 / s+2, valid if st1 / st2.
// INA_GEMM_SCHED 1 (balanced, default): p0 stages A1 of s+1, p1 A0, p2 B0, p3 B1 of s+2 -- one half-tile
//   (2 DMAs per thread) per phase; waits vmcnt(10) in p0 (B1 of s), p1 (A1 of s), p3 (A0 + B0 of s+1): every
//   half-tile has 5-6 phases between its issue and its wait.
// INA_GEMM_SCHED 0 (front-loaded): p1 A0 + B0, p2 B1, p3 A1 of s+2; waits vmcnt(10 / 12 / 12).
template <int BUF>
INA_DEVICE void kstep(f32x4_t (&acc)[8][4], Frags& f, const Stager& sg, bool full, bool st1, bool st2,
                      const StagePos& p1, const StagePos& p2, uint32_t rdA0, uint32_t rdA1, uint32_t rdB0,
                      uint32_t rdB1) {
  constexpr int OTHER = BUF ^ 1;
  const unsigned char* buf = gemm_lds + BUF * G_BUF;
  auto read_a = [&](u16x8_t (&fa)[4][2], int H) {
    const unsigned char* img = buf + H * G_HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = ldsr(img + rdA0 + i * 16 * 128);
      fa[i][1] = ldsr(img + rdA1 + i * 16 * 128);
    }
  };
  auto read_b = [&](u16x8_t (&fb)[2][2], int H) {
    const unsigned char* img = buf + (2 + H) * G_HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[j][0] = ldsr(img + rdB0 + j * 16 * 128);
      fb[j][1] = ldsr(img + rdB1 + j * 16 * 128);
    }
  };
  if constexpr (INA_GEMM_SCHED == 2) {
    // two phases of 32 MFMAs (4 barriers per K-step instead of 8):
    // X: A0 / B0 / B1 subtiles, quadrants (A0,B0) (A0,B1); stage A1 of s+1; A1 of s must land before Y
    read_b(f.b0, 0);
    read_b(f.b1, 1);
    read_a(f.a0, 0);
    if (st1) sg.stage(OTHER, 1, p1.m, p1.n, p1.k);
    wait_lgkm0();
    if (full) wait_vm<8>(); else wait_vm<0>();
    barrier();
    mma_quadrant<0, 0>(acc, f.a0, f.b0);
    mma_quadrant<0, 1>(acc, f.a0, f.b1);
    barrier();
    // Y: A1 subtile, quadrants (A1,B1) (A1,B0); restage A0 / B0 / B1 (read in X) with s+2; A0 / B0 / B1 of
    // s+1 must land before its X
    read_a(f.a1, 1);
    if (st2) {
      sg.stage(BUF, 0, p2.m, p2.n, p2.k);
      sg.stage(BUF, 2, p2.m, p2.n, p2.k);
      sg.stage(BUF, 3, p2.m, p2.n, p2.k);
    }
    wait_lgkm0();
    if (full) wait_vm<8>(); else wait_vm<0>();
    barrier();
    mma_quadrant<1, 1>(acc, f.a1, f.b1);
    mma_quadrant<1, 0>(acc, f.a1, f.b0);
    barrier();
    return;
  }
  // p0: A0 / B0 subtiles; B1 of this step must have landed before p1 reads it
  read_b(f.b0, 0);
  read_a(f.a0, 0);
  if (INA_GEMM_SCHED && st1) sg.stage(OTHER, 1, p1.m, p1.n, p1.k);
  wait_lgkm0();
  if (full) wait_vm<10>(); else wait_vm<0>();
  barrier();
  mma_quadrant<0, 0>(acc, f.a0, f.b0);
  barrier();
  // p1: B1 subtile; restage A0 (+ B0) (read in p0) with step s+2; A1 must land before p2
  read_b(f.b1, 1);
  if (st2) {
    sg.stage(BUF, 0, p2.m, p2.n, p2.k);
    if (!INA_GEMM_SCHED) sg.stage(BUF, 2, p2.m, p2.n, p2.k);
  }
  wait_lgkm0();
  if (full) wait_vm<INA_GEMM_SCHED ? 10 : 12>(); else wait_vm<0>();
  barrier();
  mma_quadrant<0, 1>(acc, f.a0, f.b1);
  barrier();
  // p2: A1 subtile; restage B0 (read in p0) / B1 (read in p1)
  read_a(f.a1, 1);
  if (st2) sg.stage(BUF, INA_GEMM_SCHED ? 2 : 3, p2.m, p2.n, p2.k);
  wait_lgkm0();
  barrier();
  mma_quadrant<1, 1>(acc, f.a1, f.b1);
  barrier();
  // p3: no reads; restage B1 (read in p1) / A1 (read in p2); A0 + B0 of step s+1 must land before its p0
  if (st2) sg.stage(BUF, INA_GEMM_SCHED ? 3 : 1, p2.m, p2.n, p2.k);
  if (full) wait_vm<INA_GEMM_SCHED ? 10 : 12>(); else wait_vm<0>();
  barrier();
  mma_quadrant<1, 0>(acc, f.a1, f.b0);
  barrier();
}

// EPI_DGELU: per (row tile mt, half h) ONE 16-byte aux load per lane (the widened layout, unwidened in
// registers) instead of two 8-byte ones, all 16 of the wave's aux loads issued before the first use; d in the
// accumulator layout (bias-gradient column sums as before), stored widened.
INA_DEVICE void epilogue_dgelu(const f32x4_t (&acc)[8][4], const GemmArgs& g, int m0, int n0, int wr, int wc, int fr,
                               int fq) {
  uint4 xa[8][2];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + (mt >> 2) * 128 + wr * 64 + (mt & 3) * 16 + fr;
    const size_t mrow = (size_t)(m < g.M ? m : 0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      xa[mt][h] = *reinterpret_cast<const uint4*>(g.aux + mrow * g.ldx + n0 + h * 128 + wc * 32 + 8 * fq);
  }
  float cs[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[nt][r] = 0.f;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + (mt >> 2) * 128 + wr * 64 + (mt & 3) * 16 + fr;
    const bool ok = m < g.M;
    const size_t mrow = (size_t)(ok ? m : 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint2 ax = uint2{xa[mt][h].x, xa[mt][h].y}, ay = uint2{xa[mt][h].z, xa[mt][h].w};
      unwiden(ax, ay);
      const u16x4_t xv[2] = {__builtin_bit_cast(u16x4_t, ax), __builtin_bit_cast(u16x4_t, ay)};
      u16x4_t o[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = ok ? acc[mt][2 * h + j][r] * gelu_d(bf2f(xv[j][r])) : 0.f;
          o[j][r] = f2bf(d);
          cs[2 * h + j][r] += d;
        }
      uint2 X = __builtin_bit_cast(uint2, o[0]), Y = __builtin_bit_cast(uint2, o[1]);
      widen(X, Y);
      if (ok) *reinterpret_cast<uint4*>(g.out + mrow * g.ldo + n0 + h * 128 + wc * 32 + 8 * fq) = uint4{X.x, X.y, Y.x, Y.y};
    }
  }
  float* srow = g.slab + (size_t)(2 * (m0 / G_BM) + wr) * g.N;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    float4 sv;
    sv.x = group16_sum(cs[nt][0]);
    sv.y = group16_sum(cs[nt][1]);
    sv.z = group16_sum(cs[nt][2]);
    sv.w = group16_sum(cs[nt][3]);
    if (fr == 0) *reinterpret_cast<float4*>(srow + n0 + (nt >> 1) * 128 + wc * 32 + (nt & 1) * 16 + 4 * fq) = sv;
  }
}

// acc[mt][nt][r] = C[m0 + mrow(mt) + fr][n0 + ncol(nt) + 4 fq + r]
template <int EPI>
INA_DEVICE void epilogue(f32x4_t (&acc)[8][4], const GemmArgs& g, int m0, int n0, int wr, int wc, int fr, int fq) {
  if constexpr (EPI == EPI_DGELU) {
    epilogue_dgelu(acc, g, m0, n0, wr, wc, fr, fq);
    return;
  }
  float cs[4][4];
  f32x4_t bb[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = n0 + (nt >> 1) * 128 + wc * 32 + (nt & 1) * 16 + 4 * fq;
    bb[nt] = (EPI == EPI_GELU || EPI == EPI_PLAIN_B) ? *reinterpret_cast<const f32x4_t*>(g.bias + n)
                                                    : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[nt][r] = 0.f;
  }
  // consume the bias loads at once: a load still pending where the K loop resumes would make hipcc drain
  // vmcnt (the in-flight DMAs) at the loop head of every K-step
  if constexpr (EPI == EPI_GELU || EPI == EPI_PLAIN_B)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(bb[0]), "+v"(bb[1]), "+v"(bb[2]), "+v"(bb[3])::"memory");
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + (mt >> 2) * 128 + wr * 64 + (mt & 3) * 16 + fr;
    const bool ok = m < g.M;
    const size_t mrow = (size_t)(ok ? m : 0);
    u16x4_t xv[4];
    if constexpr (EPI == EPI_DGELU) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int n = n0 + (nt >> 1) * 128 + wc * 32 + (nt & 1) * 16 + 4 * fq;
        xv[nt] = *reinterpret_cast<const u16x4_t*>(g.aux + mrow * g.ldx + n);
      }
    }
    u16x4_t ov[4], axv[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float bv[4] = {bb[nt][0], bb[nt][1], bb[nt][2], bb[nt][3]};
      u16x4_t o, ax;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float c = acc[mt][nt][r];
        if constexpr (EPI == EPI_PLAIN || EPI == EPI_PLAIN_B) {
          o[r] = f2bf(c + bv[r]);
        } else if constexpr (EPI == EPI_GELU) {
          const float u = c + bv[r];
          ax[r] = f2bf(u);
          o[r] = f2bf(gelu_v(u));
        } else {
          const float d = ok ? c * gelu_d(bf2f(xv[nt][r])) : 0.f;
          o[r] = f2bf(d);
          cs[nt][r] += d;
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
      if (ok && (!INA_GEMM_NOSTORE || X.x == 0x7FC17FC1u))   // (diagnostic: a never-true use keeps the MFMAs)
        *reinterpret_cast<uint4*>(g.out + mrow * g.ldo + n) = uint4{X.x, X.y, Y.x, Y.y};
      if constexpr (EPI == EPI_GELU) {
        uint2 Xa = __builtin_bit_cast(uint2, axv[2 * h]), Ya = __builtin_bit_cast(uint2, axv[2 * h + 1]);
        widen(Xa, Ya);
        if (ok) *reinterpret_cast<uint4*>(g.aux + mrow * g.ldx + n) = uint4{Xa.x, Xa.y, Ya.x, Ya.y};
      }
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    float* srow = g.slab + (size_t)(2 * (m0 / G_BM) + wr) * g.N;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float4 s;
      s.x = group16_sum(cs[nt][0]);
      s.y = group16_sum(cs[nt][1]);
      s.z = group16_sum(cs[nt][2]);
      s.w = group16_sum(cs[nt][3]);
      if (fr == 0) {
        const int n = n0 + (nt >> 1) * 128 + wc * 32 + (nt & 1) * 16 + 4 * fq;
        *reinterpret_cast<float4*>(srow + n) = s;
      }
    }
  }
}

// Persistent: block b runs tiles b, b + grid, b + 2 grid, ... as ONE stream of K-steps (s = local tile * T
// + kt, buffer s & 1), so the DMA of the next tile's first two K-steps is in flight during the current
// tile's last two and its epilogue; there is one pipeline fill per block, not per tile.
// Staging of K-step s+2 during step s: p1 A0 + B0, p2 B1, p3 A1 (each one phase after its last read);
// waits: p0 vmcnt(10) (B1 of s), p1 vmcnt(12) (A1 of s), p3 vmcnt(12) (A0 + B0 of s+1): every half-tile
// has 6 phases between its DMA issue and its wait.
template <int EPI>
__global__ __launch_bounds__(G_THREADS, 1) void gemm_bf16_nt_kernel(GemmArgs g) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int NB = g.N / G_BN, MBn = (g.M + G_BM - 1) / G_BM, NT = MBn * NB;
  const int G = gridDim.x, b = blockIdx.x;
  const int T = g.K / G_BK;
  const int ntile = (NT - b + G - 1) / G;
  const int S = ntile * T;

  Stager sg;
  sg.gA = reinterpret_cast<const unsigned char*>(g.A);
  sg.gB = reinterpret_cast<const unsigned char*>(g.B);
  sg.lda2 = g.lda * 2;
  sg.ldb2 = g.ldb * 2;
  sg.M1 = g.M - 1;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 16 * w + 8 * j + (lane >> 3);
    sg.row[j] = r;
    sg.chunk[j] = ((lane & 7) ^ ((r >> 1) & 7)) * 16;
  }
  sg.dst0 = 2 * w * 1024;
  // fragment read offsets: row (l & 15) of a 16-row tile, logical chunk 4 kk + (l >> 4), swizzled
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t rdA0 = (uint32_t)((wr * 64 + fr) * 128 + ((fq ^ (fr >> 1)) * 16));
  const uint32_t rdA1 = (uint32_t)((wr * 64 + fr) * 128 + (((4 + fq) ^ (fr >> 1)) * 16));
  const uint32_t rdB0 = (uint32_t)((wc * 32 + fr) * 128 + ((fq ^ (fr >> 1)) * 16));
  const uint32_t rdB1 = (uint32_t)((wc * 32 + fr) * 128 + (((4 + fq) ^ (fr >> 1)) * 16));

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  Frags f;

  // current tile (compute) and the stream positions one and two steps ahead (staging)
  int jt = 0, kt = 0, m0, n0;
  tile_coords(b, NT, NB, m0, n0);
  StagePos p1{m0, n0, 0}, p2{m0, n0, 0};
  int j2 = 0;
  auto adv2 = [&]() {   // p1 <- p2, p2 <- the next K-step of the stream
    p1 = p2;
    if (++p2.k == T) {
      p2.k = 0;
      ++j2;
      if (j2 < ntile) tile_coords(b + j2 * G, NT, NB, p2.m, p2.n);
    }
  };
  // prologue: step 0 (A0 B0 B1 A1) and step 1 (SCHED 1: A0 B0 B1, its A1 is staged in step 0's p0;
  // SCHED 0: A0 B0 B1 A1), in the order the counted waits assume
  for (int p = 0; p < 2 && p < S; ++p) {
    sg.stage(p, 0, p2.m, p2.n, p2.k);
    sg.stage(p, 2, p2.m, p2.n, p2.k);
    sg.stage(p, 3, p2.m, p2.n, p2.k);
    if (!INA_GEMM_SCHED || p == 0) sg.stage(p, 1, p2.m, p2.n, p2.k);
    adv2();
  }
  if (S > 1) wait_vm<INA_GEMM_SCHED == 2 ? 8 : (INA_GEMM_SCHED ? 10 : 12)>(); else wait_vm<0>();
  barrier();
  if (INA_GEMM_STAGGER && wr == 1) barrier();  // ping-pong: row group 1 runs one barrier behind row group 0

  for (int s = 0; s < S; s += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ss = s + u;
      if (ss < S) {
        const bool st1 = ss + 1 < S, st2 = ss + 2 < S;
        if (u == 0)
          kstep<0>(acc, f, sg, st2, st1, st2, p1, p2, rdA0, rdA1, rdB0, rdB1);
        else
          kstep<1>(acc, f, sg, st2, st1, st2, p1, p2, rdA0, rdA1, rdB0, rdB1);
        adv2();
        if (++kt == T) {
          epilogue<EPI>(acc, g, m0, n0, wr, wc, fr, fq);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          kt = 0;
          if (++jt < ntile) tile_coords(b + jt * G, NT, NB, m0, n0);
        }
      }
    }
  }
  if (INA_GEMM_STAGGER && wr == 0) barrier();  // balance the barrier counts of the two row groups
}

template <int EPI>
int launch_gemm(const GemmArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_bf16_nt_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            G_LDS) != hipSuccess)
      return 2;
    attr = true;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      return 3;
    ncu &= ~7;  // a multiple of 8: every block's tiles stay on its XCD (tile_coords)
  }
  const long tiles = (long)((a.M + G_BM - 1) / G_BM) * (a.N / G_BN);
  const long grid = tiles < ncu ? tiles : ncu;  // persistent: one workgroup per CU
  hipLaunchKernelGGL(gemm_bf16_nt_kernel<EPI>, dim3((unsigned)grid), dim3(G_THREADS), G_LDS, st, a);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace

namespace ina {

int gemm_bf16_nt(const void* A, int lda, const void* B, int ldb, int M, int N, int K, const float* bias, void* out,
                 int ldo, void* aux, int ldx, float* slab, int epi, hipStream_t st) {
  if (M <= 0 || N <= 0 || N % G_BN != 0 || K < G_BK || K % G_BK != 0) return 1;
  // 16-byte epilogue stores (widen): ldo / ldx multiples of 8 elements, 16-byte aligned bases
  if (lda % 8 != 0 || ldb % 8 != 0 || ldo % 8 != 0 || lda < K || ldb < K || ldo < N) return 1;
  if (((uintptr_t)out & 15) != 0 || ((uintptr_t)aux & 15) != 0) return 1;
  // 32-bit byte offsets of the DMA sources
  if ((long)M * lda * 2 >= (1L << 31) || (long)N * ldb * 2 >= (1L << 31)) return 1;
  if (epi != EPI_PLAIN && (aux == nullptr || ldx % 8 != 0 || ldx < N)) return 1;
  if (epi == EPI_GELU && bias == nullptr) return 1;
  if (epi == EPI_DGELU && slab == nullptr) return 1;
  GemmArgs a{(const unsigned short*)A, (const unsigned short*)B, bias, (unsigned short*)out, (unsigned short*)aux,
             slab, M, N, K, lda, ldb, ldo, ldx};
  switch (epi) {
    case EPI_PLAIN: return bias != nullptr ? launch_gemm<EPI_PLAIN_B>(a, st) : launch_gemm<EPI_PLAIN>(a, st);
    case EPI_GELU: return launch_gemm<EPI_GELU>(a, st);
    case EPI_DGELU: return launch_gemm<EPI_DGELU>(a, st);
    default: return 1;
  }
}

}  // namespace ina
