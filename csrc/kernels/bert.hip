// BERT encoder kernels for gfx950 (north-star BERT path; BASELINE config
// "FewRel 10-way 5-shot with BERT-base encoder").  The reference has no BERT; the math is standard
// post-LN BERT and the oracle is models/bert.py.
//
//  * embed_ln     : x = word[id] + pos[t] + type[0];  y = LN(x) (+ hidden dropout)      fwd / bwd
//  * ln_res       : y = LN(res + dropout(a))  (attention-output and FFN-output sublayers)  fwd / bwd
//  * bias_gelu    : y = gelu(x + b)  (erf form), db summed per block                        fwd / bwd
//  * mha          : fused multi-head attention for one (sequence, head) per workgroup with the
//                   whole sequence (L <= 128) resident in LDS; MFMA 16x16x32 bf16 for all
//                   products; softmax in registers; attention-probability dropout from the
//                   counter hash; backward recomputes P from the saved log-sum-exp.
//
// Row kernels (LN, embed) put one row on one wave: lane l owns columns 256c + 4l .. +3 (c < NCH),
// 8-byte bf16 loads/stores, wave-shuffle reductions; hidden width HD = 256 * NCH.
//
// MHA layouts (lane l: n = l & 15, g = l >> 4; MFMA C[row 4g + r][col n]):
//  forward ("query on the lane"): S^T = K Q^T tiles (A = K rows from LDS, B = the query's 16-B
//    row slices kept in registers), so the softmax over keys is in-register + a 4-lane-group
//    shuffle; O^T = V^T P^T takes the P^T accumulators directly as the B operand (kmap key order)
//    and V^T from LDS.
//  backward ("key on the lane"): each wave owns key tiles; S = Q K^T and dP = dO V^T have the key
//    on the lane, so dV^T = dO^T P' and dK^T = Q^T dS take P'/dS accumulators as B operands (q in
//    kmap order, dO^T / Q^T from LDS); dS crosses LDS once for dQ^T = K^T dS^T.
#include <cstdlib>

#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr float LN_EPS = 1e-12f;

#define INA_PRAGMA(x) _Pragma(#x)
#define INA_UNROLL(n) INA_PRAGMA(unroll n)
#ifndef INA_MHA_KTU
#define INA_MHA_KTU 1   // mha_bwd key-tile loop unroll (A/B)
#endif
#ifndef INA_MHA_QPU
#define INA_MHA_QPU 1   // mha_bwd query-pair loop unroll (A/B)
#endif
constexpr float LOG2E = 1.4426950408889634f;

INA_DEVICE void ld4(const unsigned short* p, float* v) {
  const u16x4_t x = *reinterpret_cast<const u16x4_t*>(p);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = bf2f(x[r]);
}
INA_DEVICE void st4(unsigned short* p, const float* v) {
  u16x4_t x;
#pragma unroll
  for (int r = 0; r < 4; ++r) x[r] = f2bf(v[r]);
  *reinterpret_cast<u16x4_t*>(p) = x;
}
INA_DEVICE float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
// One row's 4-column groups of two 16-column tiles (a0: columns 4g .. 4g+3 of tile dt, a1: the same of tile dt+1)
// -> ONE 16-byte store per lane of columns 8g .. 8g+7 (ina_common.h widen; all lanes must call it, ok masks the
// store): 16 rows x 64 B per instruction instead of two instructions of 16 rows x 32 B.  p = the row's base + 32
// columns per tile pair.
INA_DEVICE void st8w(unsigned short* p, int g, const float* a0, const float* a1, bool ok) {
  u16x4_t x, y;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    x[r] = f2bf(a0[r]);
    y[r] = f2bf(a1[r]);
  }
  uint2 X = __builtin_bit_cast(uint2, x), Y = __builtin_bit_cast(uint2, y);
  widen(X, Y);
  if (ok) *reinterpret_cast<uint4*>(p + 8 * g) = uint4{X.x, X.y, Y.x, Y.y};
}

// --------------------------------------------------------------------------------------------
// LN(res + dropout(a))
// --------------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void ln_res_fwd_kernel(const unsigned short* __restrict__ a,
                                                         const unsigned short* __restrict__ res,
                                                         const float* __restrict__ gam, const float* __restrict__ bet,
                                                         unsigned short* __restrict__ y, float* __restrict__ stats,
                                                         int T, uint32_t salt, uint32_t thr, float inv_kp, int drop) {
  constexpr int HD = 256 * NCH;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= T) return;
  const size_t base = (size_t)row * HD;
  float x[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = 256 * c + 4 * lane;
    float av[4], rv[4];
    ld4(a + base + col, av);
    ld4(res + base + col, rv);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = av[r];
      if (drop) v = dropout_keep_salted(salt, (uint32_t)(base + col + r), thr) ? v * inv_kp : 0.f;
      x[c][r] = v + rv[r];
      s += x[c][r];
    }
  }
  const float mean = wave_sum(s) * (1.f / HD);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = x[c][r] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / HD) + LN_EPS);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = 256 * c + 4 * lane;
    const float4 gv = ld4f(gam + col), bv = ld4f(bet + col);
    float o[4] = {(x[c][0] - mean) * rstd * gv.x + bv.x, (x[c][1] - mean) * rstd * gv.y + bv.y,
                  (x[c][2] - mean) * rstd * gv.z + bv.z, (x[c][3] - mean) * rstd * gv.w + bv.w};
    st4(y + base + col, o);
  }
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = rstd;
  }
}

// dres = dLN/dx (bf16), da = dres * dropout mask / kp (bf16), slab[block] = [dgamma | dbeta]
template <int NCH>
__global__ __launch_bounds__(256) void ln_res_bwd_kernel(
    const unsigned short* __restrict__ dy, const unsigned short* __restrict__ a, const unsigned short* __restrict__ res,
    const float* __restrict__ gam, const float* __restrict__ stats, unsigned short* __restrict__ dres,
    unsigned short* __restrict__ da, float* __restrict__ slab, int T, uint32_t salt, uint32_t thr, float inv_kp,
    int drop) {
  constexpr int HD = 256 * NCH;
  __shared__ float red[4][3][HD];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // slab rows: d gamma, d beta, and the column sums of da (the bias gradient of the projection that
  // produced a: one pass instead of a separate reduction over the [T, HD] activation gradient)
  float dg[NCH][4], db[NCH][4], dd[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) dg[c][r] = db[c][r] = dd[c][r] = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < T; row += gridDim.x * 4) {
    const size_t base = (size_t)row * HD;
    const float mean = stats[2 * row], rstd = stats[2 * row + 1];
    float xh[NCH][4], dyg[NCH][4], dyv[NCH][4];
    bool keep[NCH][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = 256 * c + 4 * lane;
      float av[4], rv[4];
      ld4(a + base + col, av);
      ld4(res + base + col, rv);
      ld4(dy + base + col, dyv[c]);
      const float4 gv = ld4f(gam + col);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        keep[c][r] = !drop || dropout_keep_salted(salt, (uint32_t)(base + col + r), thr);
        const float v = drop ? (keep[c][r] ? av[r] * inv_kp : 0.f) : av[r];
        xh[c][r] = (v + rv[r] - mean) * rstd;
        dyg[c][r] = dyv[c][r] * gg[r];
        s1 += dyg[c][r];
        s2 += dyg[c][r] * xh[c][r];
        dg[c][r] += dyv[c][r] * xh[c][r];
        db[c][r] += dyv[c][r];
      }
    }
    const float m1 = wave_sum(s1) * (1.f / HD), m2 = wave_sum(s2) * (1.f / HD);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = 256 * c + 4 * lane;
      float dx[4], dav[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dx[r] = rstd * (dyg[c][r] - m1 - xh[c][r] * m2);
        dav[r] = drop ? (keep[c][r] ? dx[r] * inv_kp : 0.f) : dx[r];
        dd[c][r] += round_bf(dav[r]);   // the stored bf16 values
      }
      st4(dres + base + col, dx);
      st4(da + base + col, dav);
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[wave][0][256 * c + 4 * lane + r] = dg[c][r];
      red[wave][1][256 * c + 4 * lane + r] = db[c][r];
      red[wave][2][256 * c + 4 * lane + r] = dd[c][r];
    }
  __syncthreads();
  float* out = slab + (size_t)blockIdx.x * 3 * HD;
  for (int i = threadIdx.x; i < 3 * HD; i += 256) {
    const int k = i / HD, col = i - k * HD;
    out[i] = red[0][k][col] + red[1][k][col] + red[2][k][col] + red[3][k][col];
  }
}

// --------------------------------------------------------------------------------------------
// embeddings: x = word[id] + pos[t] + type[0];  y = dropout(LN(x))
// --------------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void embed_ln_fwd_kernel(
    const int* __restrict__ inst, const int* __restrict__ ids_all, int S, int L, const float* __restrict__ wemb,
    const float* __restrict__ pemb, const float* __restrict__ temb, const float* __restrict__ gam,
    const float* __restrict__ bet, unsigned short* __restrict__ y, float* __restrict__ stats, uint32_t salt,
    uint32_t thr, float inv_kp, int drop) {
  constexpr int HD = 256 * NCH;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= S * L) return;
  const int s = row / L, t = row - s * L;
  const int id = ids_all[(size_t)inst[s] * L + t];
  const size_t base = (size_t)row * HD;
  float x[NCH][4];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = 256 * c + 4 * lane;
    const float4 w = ld4f(wemb + (size_t)id * HD + col), p = ld4f(pemb + (size_t)t * HD + col),
                 ty = ld4f(temb + col);
    x[c][0] = w.x + p.x + ty.x;
    x[c][1] = w.y + p.y + ty.y;
    x[c][2] = w.z + p.z + ty.z;
    x[c][3] = w.w + p.w + ty.w;
    sum += x[c][0] + x[c][1] + x[c][2] + x[c][3];
  }
  const float mean = wave_sum(sum) * (1.f / HD);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) q += (x[c][r] - mean) * (x[c][r] - mean);
  const float rstd = rsqrtf(wave_sum(q) * (1.f / HD) + LN_EPS);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = 256 * c + 4 * lane;
    const float4 gv = ld4f(gam + col), bv = ld4f(bet + col);
    const float gg[4] = {gv.x, gv.y, gv.z, gv.w}, bb[4] = {bv.x, bv.y, bv.z, bv.w};
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      o[r] = (x[c][r] - mean) * rstd * gg[r] + bb[r];
      if (drop) o[r] = dropout_keep_salted(salt, (uint32_t)(base + col + r), thr) ? o[r] * inv_kp : 0.f;
    }
    st4(y + base + col, o);
  }
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = rstd;
  }
}

// dx (fp32 [T, HD], the gradient of the summed embedding; the caller scatters it into the word /
// position / type tables) and slab[block] = [dgamma | dbeta]
template <int NCH>
__global__ __launch_bounds__(256) void embed_ln_bwd_kernel(
    const unsigned short* __restrict__ dy, const int* __restrict__ inst, const int* __restrict__ ids_all, int S,
    int L, const float* __restrict__ wemb, const float* __restrict__ pemb, const float* __restrict__ temb,
    const float* __restrict__ gam, const float* __restrict__ stats, float* __restrict__ dx, float* __restrict__ slab,
    uint32_t salt, uint32_t thr, float inv_kp, int drop) {
  constexpr int HD = 256 * NCH;
  __shared__ float red[4][2][HD];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float dg[NCH][4], db[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) dg[c][r] = db[c][r] = 0.f;
  const int T = S * L;
  for (int row = blockIdx.x * 4 + wave; row < T; row += gridDim.x * 4) {
    const int s = row / L, t = row - s * L;
    const int id = ids_all[(size_t)inst[s] * L + t];
    const size_t base = (size_t)row * HD;
    const float mean = stats[2 * row], rstd = stats[2 * row + 1];
    float xh[NCH][4], dyg[NCH][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = 256 * c + 4 * lane;
      const float4 w = ld4f(wemb + (size_t)id * HD + col), p = ld4f(pemb + (size_t)t * HD + col),
                   ty = ld4f(temb + col), gv = ld4f(gam + col);
      const float xv[4] = {w.x + p.x + ty.x, w.y + p.y + ty.y, w.z + p.z + ty.z, w.w + p.w + ty.w};
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
      float dyv[4];
      ld4(dy + base + col, dyv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (drop) dyv[r] = dropout_keep_salted(salt, (uint32_t)(base + col + r), thr) ? dyv[r] * inv_kp : 0.f;
        xh[c][r] = (xv[r] - mean) * rstd;
        dyg[c][r] = dyv[r] * gg[r];
        s1 += dyg[c][r];
        s2 += dyg[c][r] * xh[c][r];
        dg[c][r] += dyv[r] * xh[c][r];
        db[c][r] += dyv[r];
      }
    }
    const float m1 = wave_sum(s1) * (1.f / HD), m2 = wave_sum(s2) * (1.f / HD);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = 256 * c + 4 * lane;
      float4 o;
      o.x = rstd * (dyg[c][0] - m1 - xh[c][0] * m2);
      o.y = rstd * (dyg[c][1] - m1 - xh[c][1] * m2);
      o.z = rstd * (dyg[c][2] - m1 - xh[c][2] * m2);
      o.w = rstd * (dyg[c][3] - m1 - xh[c][3] * m2);
      *reinterpret_cast<float4*>(dx + base + col) = o;
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[wave][0][256 * c + 4 * lane + r] = dg[c][r];
      red[wave][1][256 * c + 4 * lane + r] = db[c][r];
    }
  __syncthreads();
  float* out = slab + (size_t)blockIdx.x * 2 * HD;
  for (int i = threadIdx.x; i < 2 * HD; i += 256) {
    const int k = i / HD, col = i - k * HD;
    out[i] = red[0][k][col] + red[1][k][col] + red[2][k][col] + red[3][k][col];
  }
}

// --------------------------------------------------------------------------------------------
// bias + GELU (erf form)
// --------------------------------------------------------------------------------------------
INA_DEVICE float gelu_f(float u) { return 0.5f * u * (1.f + erff(u * 0.70710678118654752f)); }
INA_DEVICE float gelu_grad(float u) {
  return 0.5f * (1.f + erff(u * 0.70710678118654752f)) + u * 0.3989422804014327f * __expf(-0.5f * u * u);
}

// x, y: [T, I] bf16 row-major; I % 8 == 0.  Grid-stride over 8-element chunks.
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const unsigned short* __restrict__ x,
                                                            const float* __restrict__ b,
                                                            unsigned short* __restrict__ y, long nchunks, int I) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nchunks; i += (long)gridDim.x * 256) {
    const long e0 = i * 8;
    const int col = (int)(e0 % I);
    const u16x8_t v = *reinterpret_cast<const u16x8_t*>(x + e0);
    const float4 b0 = ld4f(b + col), b1 = ld4f(b + col + 4);
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    u16x8_t o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(gelu_f(bf2f(v[j]) + bb[j]));
    *reinterpret_cast<u16x8_t*>(y + e0) = o;
  }
}

// dx = dy * gelu'(x + b); slab[block][I] = column sums of dx over the block's rows.
// Thread t owns column chunks t, t + 256, ... (< I/8, at most CPT of them); blocks stride rows.
template <int CPT>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const unsigned short* __restrict__ dy,
                                                            const unsigned short* __restrict__ x,
                                                            const float* __restrict__ b, unsigned short* __restrict__ dx,
                                                            float* __restrict__ slab, int T, int I) {
  const int nch = I / 8;
  float acc[CPT][8];
  float bb[CPT][8];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int ch = threadIdx.x + 256 * k;
    const int col = (ch < nch ? ch : 0) * 8;
    const float4 b0 = ld4f(b + col), b1 = ld4f(b + col + 4);
    bb[k][0] = b0.x; bb[k][1] = b0.y; bb[k][2] = b0.z; bb[k][3] = b0.w;
    bb[k][4] = b1.x; bb[k][5] = b1.y; bb[k][6] = b1.z; bb[k][7] = b1.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  }
  for (int row = blockIdx.x; row < T; row += gridDim.x) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int ch = threadIdx.x + 256 * k;
      if (ch < nch) {
        const size_t e0 = (size_t)row * I + ch * 8;
        const u16x8_t gv = *reinterpret_cast<const u16x8_t*>(dy + e0);
        const u16x8_t xv = *reinterpret_cast<const u16x8_t*>(x + e0);
        u16x8_t o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(gv[j]) * gelu_grad(bf2f(xv[j]) + bb[k][j]);
          o[j] = f2bf(d);
          acc[k][j] += d;
        }
        *reinterpret_cast<u16x8_t*>(dx + e0) = o;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int ch = threadIdx.x + 256 * k;
    if (ch < nch) {
      float* o = slab + (size_t)blockIdx.x * I + ch * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = acc[k][j];
    }
  }
}

// Balanced variant for R * (I/8) == 256 * NPT (I = 3072: R = 2, NPT = 3; I = 768: R = 8, NPT = 3):
// a block iteration covers R rows as R*I/8 chunks and thread t owns chunks t + 256m, so every thread
// is busy and issues all 2*NPT 16-byte loads before consuming any.  A thread's chunks keep their
// columns across iterations (the block strides R rows); the R row-slot partials of a column are
// summed in fixed slot order through LDS.
template <int NPT>
__global__ __launch_bounds__(256) void bias_gelu_bwd_bal_kernel(const unsigned short* __restrict__ dy,
                                                                const unsigned short* __restrict__ x,
                                                                const float* __restrict__ b,
                                                                unsigned short* __restrict__ dx,
                                                                float* __restrict__ slab, int T, int I, int R) {
  extern __shared__ float cs[];   // [R][I]
  const int nch = I / 8;
  int rin[NPT], col[NPT];
  float acc[NPT][8], bb[NPT][8];
#pragma unroll
  for (int m = 0; m < NPT; ++m) {
    const int c = threadIdx.x + 256 * m;
    rin[m] = c / nch;
    col[m] = (c - rin[m] * nch) * 8;
    const float4 b0 = ld4f(b + col[m]), b1 = ld4f(b + col[m] + 4);
    bb[m][0] = b0.x; bb[m][1] = b0.y; bb[m][2] = b0.z; bb[m][3] = b0.w;
    bb[m][4] = b1.x; bb[m][5] = b1.y; bb[m][6] = b1.z; bb[m][7] = b1.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[m][j] = 0.f;
  }
  for (int row0 = blockIdx.x * R; row0 < T; row0 += gridDim.x * R) {
    u16x8_t gv[NPT], xv[NPT];
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int row = row0 + rin[m] < T ? row0 + rin[m] : T - 1;
      const size_t e0 = (size_t)row * I + col[m];
      gv[m] = *reinterpret_cast<const u16x8_t*>(dy + e0);
      xv[m] = *reinterpret_cast<const u16x8_t*>(x + e0);
    }
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      if (row0 + rin[m] < T) {
        u16x8_t o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(gv[m][j]) * gelu_grad(bf2f(xv[m][j]) + bb[m][j]);
          o[j] = f2bf(d);
          acc[m][j] += d;
        }
        *reinterpret_cast<u16x8_t*>(dx + (size_t)(row0 + rin[m]) * I + col[m]) = o;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < NPT; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[rin[m] * I + col[m] + j] = acc[m][j];
  __syncthreads();
  float* o = slab + (size_t)blockIdx.x * I;
  for (int i = threadIdx.x; i < I; i += 256) {
    float v = cs[i];
    for (int r = 1; r < R; ++r) v += cs[r * I + i];
    o[i] = v;
  }
}

// --------------------------------------------------------------------------------------------
// fused multi-head attention, head dim 64, L <= 128
// --------------------------------------------------------------------------------------------
constexpr int HDIM = 64;
constexpr int KSTR = HDIM + 8;  // LDS row stride (bf16) of row-major [key][d] images

// Attention-probability dropout: ONE hash per pair of adjacent keys.  Element (row, key), row = (s nh + h) L + q,
// keeps iff 16-bit half (key & 1) of mix(pidx * C + salt), pidx = (row << 6) | (key >> 1), is < thr >> 16 (keep
// rate floor(kp 2^16) / 2^16; L <= 128).  pidx * C splits into a per-row / per-lane base plus compile-time
// multiples of C, so the forward costs one add + the mix per PAIR.  Bit-identical to models/bert.py::attn_keep_mask.
constexpr uint32_t ATTN_C = 0x6C8E9CF5u;
INA_DEVICE uint32_t attn_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x;
}

INA_DEVICE u16x8_t ld8(const unsigned short* p) { return *reinterpret_cast<const u16x8_t*>(p); }
INA_DEVICE u16x8_t zero8() { return u16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
INA_DEVICE u16x8_t cat_tr(const s16x4_t& a, const s16x4_t& b) {
  return u16x8_t{(unsigned short)a[0], (unsigned short)a[1], (unsigned short)a[2], (unsigned short)a[3],
                 (unsigned short)b[0], (unsigned short)b[1], (unsigned short)b[2], (unsigned short)b[3]};
}

// qkv: [T, 3*HDm] bf16, HDm = nh*64; token row of (s, t) = s*L + t.  ctx: [T, HDm] bf16.
// lse: [S, nh, LP] fp32 (log2-domain log-sum-exp of the scaled scores).  mask_all: [NI, L] int.
template <int LP, int NWV>
__global__ __launch_bounds__(64 * NWV) void mha_fwd_kernel(const unsigned short* __restrict__ qkv,
                                                      const int* __restrict__ inst, const int* __restrict__ mask_all,
                                                      int S, int L, int nh, unsigned short* __restrict__ ctx,
                                                      float* __restrict__ lse, uint32_t salt, uint32_t thr,
                                                      float inv_kp, int drop) {
  constexpr int NT = LP / 16;        // key / query tiles
  __shared__ __attribute__((aligned(16))) unsigned short Ks[LP * KSTR];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[LP * KSTR];   // V^T operands via tr_read
  __shared__ float madd[LP];
  const int s = blockIdx.x / nh, hh = blockIdx.x - s * nh;
  const int HDm = nh * HDIM, ROW = 3 * HDm;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = lane & 15, g = lane >> 4;
  const size_t tok0 = (size_t)s * L;
  const unsigned short* kbase = qkv + tok0 * ROW + HDm + hh * HDIM;
  const unsigned short* vbase = qkv + tok0 * ROW + 2 * HDm + hh * HDIM;
  // stage K and V rows (rows >= L are zero), key mask
  constexpr int NTH = 64 * NWV;
  {
    constexpr int NU = (LP * 8 + NTH - 1) / NTH;
    u16x8_t kv[NU], vv[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = min(threadIdx.x + NTH * u, LP * 8 - 1);
      const int k = i >> 3, c = (i & 7) * 8;
      const size_t off = (size_t)(k < L ? k : 0) * ROW + c;
      kv[u] = ld8(kbase + off);
      vv[u] = ld8(vbase + off);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = threadIdx.x + NTH * u;
      if (i >= LP * 8) break;
      const int k = i >> 3, c = (i & 7) * 8;
      if (k >= L) kv[u] = vv[u] = zero8();
      *reinterpret_cast<u16x8_t*>(&Ks[k * KSTR + c]) = kv[u];
      *reinterpret_cast<u16x8_t*>(&Vs[k * KSTR + c]) = vv[u];
    }
  }
  const int* mrow = mask_all + (size_t)inst[s] * L;
  for (int k = threadIdx.x; k < LP; k += NTH) madd[k] = (k < L && mrow[k < L ? k : 0] > 0) ? 0.f : -INFINITY;
  __syncthreads();
  const float c2 = 0.125f * LOG2E;  // 1/sqrt(64) in the log2 domain
#pragma unroll 1
  for (int qt = wave; qt < NT; qt += NWV) {
    const int q = 16 * qt + n;
    const bool qok = q < L;
    const unsigned short* qrow = qkv + (tok0 + (qok ? q : 0)) * ROW + hh * HDIM;
    u16x8_t qf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[ks] = ld8(qrow + 32 * ks + 8 * g);
      if (!qok) qf[ks] = zero8();
    }
    float sc[NT][4];
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        acc = mfma_bf16(ld8(&Ks[(16 * kt + n) * KSTR + 32 * ks + 8 * g]), qf[ks], acc);
      const float4 ma = *reinterpret_cast<const float4*>(&madd[16 * kt + 4 * g]);
      sc[kt][0] = acc[0] * c2 + ma.x;
      sc[kt][1] = acc[1] * c2 + ma.y;
      sc[kt][2] = acc[2] * c2 + ma.z;
      sc[kt][3] = acc[3] * c2 + ma.w;
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, sc[kt][r]);
    }
    m = cross_group_max(m);
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[kt][r] = __builtin_amdgcn_exp2f(sc[kt][r] - m);   // arguments <= 0: v_exp_f32, no range fix-up
        l += sc[kt][r];
      }
    l = cross_group_sum(l);
    // the dropout scale 1 / kp goes into the output scaling with 1 / l
    const float inv_l = (drop ? inv_kp : 1.f) / l;
    if (drop) {
      // pairs (4g + 2hr, +1) of key tile kt: pidx = (row << 6) + 8 kt + 2 g + hr
      const uint32_t thr16 = thr >> 16;
      const uint32_t hb = ((((uint32_t)(s * nh + hh) * L + q) << 6) + 2 * g) * ATTN_C + salt;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) {
          const uint32_t x = attn_mix(hb + (uint32_t)(8 * kt + hr) * ATTN_C);
          if ((x & 0xFFFFu) >= thr16) sc[kt][2 * hr] = 0.f;
          if ((x >> 16) >= thr16) sc[kt][2 * hr + 1] = 0.f;
        }
    }
    // O^T = V^T P^T: B operand = P^T accumulators (k-step ks2 covers key tiles 2ks2, 2ks2+1)
    u16x8_t pf[NT / 2];
#pragma unroll
    for (int k2 = 0; k2 < NT / 2; ++k2)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[k2][j] = f2bf(sc[2 * k2 + (j >> 2)][j & 3]);
    unsigned short* orow = ctx + (tok0 + (qok ? q : 0)) * HDm + hh * HDIM;
    float o[4][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k2 = 0; k2 < NT / 2; ++k2) {
        // A = V^T rows d = 16dt + n, k = keys in kmap order (32k2 + 4g + j, 32k2 + 16 + 4g + j)
        const unsigned short* vr = &Vs[(32 * k2 + 4 * g + (n >> 2)) * KSTR + 16 * dt + 4 * (n & 3)];
        acc = mfma_bf16(cat_tr(tr_read(vr), tr_read(vr + 16 * KSTR)), pf[k2], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] = acc[r] * inv_l;
    }
    st8w(orow, g, o[0], o[1], qok);
    st8w(orow + 32, g, o[2], o[3], qok);
    if (g == 0) lse[((size_t)s * nh + hh) * LP + q] = m + __log2f(l);
  }
}

// dqkv: [T, 3*HDm] bf16 (dQ | dK | dV), fully written (rows of tokens < L).
// bsum (optional): [S * nh][3][64] column sums of this block's stored dQ / dK / dV (the QKV bias
// gradient before the sum over sequences; one small slab instead of a [T, 3*HDm] reduction).
template <int LP, int NWV>
__global__ __launch_bounds__(64 * NWV) void mha_bwd_kernel(const unsigned short* __restrict__ qkv,
                                                      const unsigned short* __restrict__ ctx,
                                                      const unsigned short* __restrict__ dctx,
                                                      const float* __restrict__ lse, const int* __restrict__ inst,
                                                      const int* __restrict__ mask_all, int S, int L, int nh,
                                                      unsigned short* __restrict__ dqkv, uint32_t salt, uint32_t thr,
                                                      float inv_kp, int drop, float* __restrict__ bsum) {
  constexpr int NT = LP / 16;
  // Every operand image is stored row-major as it arrives (16-byte / 8-byte LDS stores) and the
  // transposed operands are read with the hardware transpose (tr_read).  Strides: 4 consecutive rows
  // land in disjoint 8-dword bank windows for the tr_read pattern.
  constexpr int DSTR = HDIM + 8;     // [q][d] / [key][d] images
  constexpr int SSTR = LP + 16;      // dS^T [key][q]
  // region A: Q and dO (phase 1), then K (phase 2)
  __shared__ __attribute__((aligned(16))) unsigned short TA[2 * LP * DSTR];
  __shared__ __attribute__((aligned(16))) unsigned short dSt[LP * SSTR];
  __shared__ float delta[LP];
  __shared__ float madd[LP];
  __shared__ float lsel[LP];
  __shared__ float wsum[NWV][3][HDIM];   // per-wave column sums (dQ | dK | dV), summed in fixed order
  constexpr int NTH = 64 * NWV;
  unsigned short* Qn = TA;
  unsigned short* dOn = TA + LP * DSTR;
  unsigned short* Kn = TA;
  const int s = blockIdx.x / nh, hh = blockIdx.x - s * nh;
  const int HDm = nh * HDIM, ROW = 3 * HDm;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = lane & 15, g = lane >> 4;
  const size_t tok0 = (size_t)s * L;
  const unsigned short* qb = qkv + tok0 * ROW + hh * HDIM;
  const unsigned short* kb = qb + HDm;
  const unsigned short* vb = qb + 2 * HDm;
  const unsigned short* ob = ctx + tok0 * HDm + hh * HDIM;
  const unsigned short* gb = dctx + tok0 * HDm + hh * HDIM;
  const float* lrow = lse + ((size_t)s * nh + hh) * LP;
  // phase 0: Q, dO images; delta = rowsum(dO * O); key mask.  All loads of a thread are issued
  // before any is consumed (one memory latency per phase, not one per row).
  {
    constexpr int NU = (LP * 8 + NTH - 1) / NTH;   // chunk i >= 8 LP: clamped load, no store
    u16x8_t qv[NU], dv[NU], ov[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = min(threadIdx.x + NTH * u, LP * 8 - 1);
      const int q = i >> 3, c = (i & 7) * 8;
      const int qc = q < L ? q : 0;
      qv[u] = ld8(qb + (size_t)qc * ROW + c);
      dv[u] = ld8(gb + (size_t)qc * HDm + c);
      ov[u] = ld8(ob + (size_t)qc * HDm + c);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = threadIdx.x + NTH * u;
      if (i >= LP * 8) break;   // (wave-uniform for NTH <= 8 LP; else the tail wave's lanes)
      const int q = i >> 3, c = (i & 7) * 8;
      const bool ok = q < L;
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) d += bf2f(dv[u][j]) * bf2f(ov[u][j]);
      d += __shfl_xor(d, 1, 64);   // the 8 chunks of row q sit on 8 consecutive lanes
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 4, 64);
      if ((i & 7) == 0) delta[q] = ok ? d : 0.f;
      if (!ok) qv[u] = dv[u] = zero8();
      *reinterpret_cast<u16x8_t*>(&Qn[q * DSTR + c]) = qv[u];
      *reinterpret_cast<u16x8_t*>(&dOn[q * DSTR + c]) = dv[u];
    }
  }
  const int* mrow = mask_all + (size_t)inst[s] * L;
  for (int k = threadIdx.x; k < LP; k += NTH) {
    madd[k] = (k < L && mrow[k < L ? k : 0] > 0) ? 0.f : -INFINITY;
    lsel[k] = lrow[k];
  }
  for (int i = threadIdx.x; i < NWV * 3 * HDIM; i += NTH) (&wsum[0][0][0])[i] = 0.f;
  __syncthreads();
  // column sums (the rounded bf16 values that are stored; rows >= L add zeros): per-lane partials in registers
  // over all of the wave's tiles, then ONE 16-lane reduction per column into this wave's slot
  float csum[3][4][4];
#pragma unroll
  for (int part = 0; part < 3; ++part)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) csum[part][dt][r] = 0.f;
  auto colsum = [&](int part, int dt, const float (&v)[4], bool ok) {
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[part][dt][r] += ok ? round_bf(v[r]) : 0.f;
  };
  auto colsum_flush = [&](int part) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = group16_sum(csum[part][dt][r]);
        if (n == 0) wsum[wave][part][16 * dt + 4 * g + r] = t;
      }
  };
  const float c2 = 0.125f * LOG2E;
  const float scale = 0.125f;
  // phase 1: each wave owns key tiles kt = wave, wave + 4
INA_UNROLL(INA_MHA_KTU)
  for (int kt = wave; kt < NT; kt += NWV) {
    const int key = 16 * kt + n;
    const bool kok = key < L;
    u16x8_t kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = ld8(kb + (size_t)(kok ? key : 0) * ROW + 32 * ks + 8 * g);
      vf[ks] = ld8(vb + (size_t)(kok ? key : 0) * ROW + 32 * ks + 8 * g);
      if (!kok) kf[ks] = vf[ks] = zero8();
    }
    const float ma = madd[key];
    // dropout hash base of the lane: (((s nh + h) L + 4 g) << 6) + (key >> 1), times C, plus the salt
    const uint32_t thr16 = thr >> 16, kshift = 16u * (uint32_t)(key & 1);
    const uint32_t kbase_h = ((((uint32_t)(s * nh + hh) * L + 4 * g) << 6) + (uint32_t)(key >> 1)) * ATTN_C + salt;
    f32x4_t dV[4], dK[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dV[dt] = dK[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
INA_UNROLL(INA_MHA_QPU)
    for (int qp = 0; qp < NT / 2; ++qp) {
      float pp[2][4], ds[2][4];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int qt = 2 * qp + h2;
        // A operands: Q and dO rows of the lane's query from the LDS images (rows >= L are zero)
        const int ra = (16 * qt + n) * DSTR + 8 * g;
        f32x4_t sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sacc = mfma_bf16(ld8(Qn + ra + 32 * ks), kf[ks], sacc);
          pacc = mfma_bf16(ld8(dOn + ra + 32 * ks), vf[ks], pacc);
        }
        const float4 lq = *reinterpret_cast<const float4*>(&lsel[16 * qt + 4 * g]);
        const float4 dq = *reinterpret_cast<const float4*>(&delta[16 * qt + 4 * g]);
        const float lqa[4] = {lq.x, lq.y, lq.z, lq.w}, dqa[4] = {dq.x, dq.y, dq.z, dq.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 16 * qt + 4 * g + r;
          const float p = (q < L) ? __builtin_amdgcn_exp2f(sacc[r] * c2 + ma - lqa[r]) : 0.f;
          float z = 1.f;
          if (drop) {   // the lane's key is fixed: pidx = ((row0 + q) << 6) + (key >> 1)
            const uint32_t x = attn_mix(kbase_h + (uint32_t)(16 * qt + r) * (64u * ATTN_C));
            z = ((x >> kshift) & 0xFFFFu) < thr16 ? inv_kp : 0.f;
          }
          const float dp = pacc[r] * z;
          pp[h2][r] = p * z;
          ds[h2][r] = p * (dp - dqa[r]);
        }
      }
      u16x8_t pf, sf;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pf[j] = f2bf(pp[j >> 2][j & 3]);
        sf[j] = f2bf(ds[j >> 2][j & 3]);
      }
      // dS^T -> LDS for the dQ phase: row key, the lane's queries 32qp + {4g..4g+3, 16+4g..16+4g+3}
      {
        unsigned short* sr = &dSt[key * SSTR + 32 * qp + 4 * g];
        *reinterpret_cast<u16x4_t*>(sr) = u16x4_t{sf[0], sf[1], sf[2], sf[3]};
        *reinterpret_cast<u16x4_t*>(sr + 16) = u16x4_t{sf[4], sf[5], sf[6], sf[7]};
      }
      // dV^T += dO^T P' ; dK^T += Q^T dS   (A rows = d, k = query in kmap order: two transposed
      // reads of query rows 32qp + 4g + j and 32qp + 16 + 4g + j)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int ro = (32 * qp + 4 * g + (n >> 2)) * DSTR + 16 * dt + 4 * (n & 3);
        dV[dt] = mfma_bf16(cat_tr(tr_read(dOn + ro), tr_read(dOn + ro + 16 * DSTR)), pf, dV[dt]);
        dK[dt] = mfma_bf16(cat_tr(tr_read(Qn + ro), tr_read(Qn + ro + 16 * DSTR)), sf, dK[dt]);
      }
    }
    // outputs: dK^T / dV^T tiles -> rows of dqkv (lane: key = 16kt + n, d = 16dt + 4g + r)
    unsigned short* dk = dqkv + (tok0 + key) * ROW + HDm + hh * HDIM;
    unsigned short* dv = dk + HDm;
    float a[4][4], b[4][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[dt][r] = dK[dt][r] * scale;
        b[dt][r] = dV[dt][r];
      }
      if (bsum) {   // uniform
        colsum(1, dt, a[dt], kok);
        colsum(2, dt, b[dt], kok);
      }
    }
    st8w(dk, g, a[0], a[1], kok);
    st8w(dk + 32, g, a[2], a[3], kok);
    st8w(dv, g, b[0], b[1], kok);
    st8w(dv + 32, g, b[2], b[3], kok);
  }
  if (bsum) {
    colsum_flush(1);
    colsum_flush(2);
  }
  __syncthreads();
  // phase 2: K image into region A, then dQ^T = K^T dS^T per query tile
  {
    constexpr int NU = (LP * 8 + NTH - 1) / NTH;   // chunk i >= 8 LP: clamped load, no store
    u16x8_t kv[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = min(threadIdx.x + NTH * u, LP * 8 - 1);
      const int k = i >> 3, c = (i & 7) * 8;
      kv[u] = ld8(kb + (size_t)(k < L ? k : 0) * ROW + c);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = threadIdx.x + NTH * u;
      if (i >= LP * 8) break;
      const int k = i >> 3, c = (i & 7) * 8;
      if (k >= L) kv[u] = zero8();
      *reinterpret_cast<u16x8_t*>(&Kn[k * DSTR + c]) = kv[u];
    }
  }
  __syncthreads();
  for (int qt = wave; qt < NT; qt += NWV) {
    const int q = 16 * qt + n;
    f32x4_t acc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k2 = 0; k2 < NT / 2; ++k2) {
      // standard k order: keys 32k2 + 8g + j, j < 8 (two transposed reads of 4 key rows each)
      const int rk = 32 * k2 + 8 * g + (n >> 2);
      const unsigned short* sb = &dSt[rk * SSTR + 16 * qt + 4 * (n & 3)];
      const u16x8_t bs = cat_tr(tr_read(sb), tr_read(sb + 4 * SSTR));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const unsigned short* kr = &Kn[rk * DSTR + 16 * dt + 4 * (n & 3)];
        acc[dt] = mfma_bf16(cat_tr(tr_read(kr), tr_read(kr + 4 * DSTR)), bs, acc[dt]);
      }
    }
    unsigned short* dq = dqkv + (tok0 + q) * ROW + hh * HDIM;
    float a[4][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) a[dt][r] = acc[dt][r] * scale;
      if (bsum) colsum(0, dt, a[dt], q < L);
    }
    st8w(dq, g, a[0], a[1], q < L);
    st8w(dq + 32, g, a[2], a[3], q < L);
  }
  if (bsum) {
    colsum_flush(0);
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * HDIM; i += NTH) {
      const float* w = &wsum[0][0][0] + i;
      float acc = 0.f;
#pragma unroll
      for (int v = 0; v < NWV; ++v) acc += w[v * 3 * HDIM];   // fixed order
      bsum[(size_t)blockIdx.x * 3 * HDIM + i] = acc;
    }
  }
}

}  // namespace

// --------------------------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------------------------
namespace ina {

#define INA_NCH_DISPATCH(HD, CALL) \
  switch ((HD) / 256) {            \
    case 1: CALL(1); break;        \
    case 2: CALL(2); break;        \
    case 3: CALL(3); break;        \
    case 4: CALL(4); break;        \
    default: return -1;            \
  }

int ln_res_fwd(const BertLnArgs& a, hipStream_t st) {
  const int grid = (a.T + 3) / 4;
#define CALL(NC)                                                                                               \
  hipLaunchKernelGGL(ln_res_fwd_kernel<NC>, dim3(grid), dim3(256), 0, st, (const unsigned short*)a.a,         \
                     (const unsigned short*)a.res, a.gamma, a.beta, (unsigned short*)a.y, a.stats, a.T, a.salt, \
                     a.thr, a.inv_kp, a.drop)
  INA_NCH_DISPATCH(a.HD, CALL)
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

int ln_res_bwd(const BertLnArgs& a, hipStream_t st) {
#define CALL(NC)                                                                                                 \
  hipLaunchKernelGGL(ln_res_bwd_kernel<NC>, dim3(a.blocks), dim3(256), 0, st, (const unsigned short*)a.dy,      \
                     (const unsigned short*)a.a, (const unsigned short*)a.res, a.gamma, a.stats,                \
                     (unsigned short*)a.dres, (unsigned short*)a.da, a.slab, a.T, a.salt, a.thr, a.inv_kp, a.drop)
  INA_NCH_DISPATCH(a.HD, CALL)
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

int embed_ln_fwd(const BertEmbArgs& a, hipStream_t st) {
  const int grid = (a.S * a.L + 3) / 4;
#define CALL(NC)                                                                                               \
  hipLaunchKernelGGL(embed_ln_fwd_kernel<NC>, dim3(grid), dim3(256), 0, st, a.inst, a.ids, a.S, a.L, a.wemb,  \
                     a.pemb, a.temb, a.gamma, a.beta, (unsigned short*)a.y, a.stats, a.salt, a.thr, a.inv_kp, \
                     a.drop)
  INA_NCH_DISPATCH(a.HD, CALL)
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

int embed_ln_bwd(const BertEmbArgs& a, hipStream_t st) {
#define CALL(NC)                                                                                                \
  hipLaunchKernelGGL(embed_ln_bwd_kernel<NC>, dim3(a.blocks), dim3(256), 0, st, (const unsigned short*)a.dy,  \
                     a.inst, a.ids, a.S, a.L, a.wemb, a.pemb, a.temb, a.gamma, a.stats, a.dx, a.slab, a.salt, \
                     a.thr, a.inv_kp, a.drop)
  INA_NCH_DISPATCH(a.HD, CALL)
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

int bias_gelu_fwd(const void* x, const float* b, void* y, long T, int I, hipStream_t st) {
  const long nchunks = T * (long)I / 8;
  long grid = (nchunks + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3((unsigned)grid), dim3(256), 0, st, (const unsigned short*)x, b,
                     (unsigned short*)y, nchunks, I);
  INA_CHECK_LAUNCH();
  return 0;
}

int bias_gelu_bwd(const void* dy, const void* x, const float* b, void* dx, float* slab, int T, int I, int blocks,
                  hipStream_t st) {
  const int nch = I / 8;
  // balanced variant: R rows per block iteration with R * nch == 3 * 256 and an [R][I] fp32 LDS slab
  if ((3 * 256) % nch == 0) {   // LDS R * I * 4 = 3 * 256 * 32 bytes
    const int R = 3 * 256 / nch;
    hipLaunchKernelGGL(bias_gelu_bwd_bal_kernel<3>, dim3(blocks), dim3(256), (size_t)R * I * sizeof(float), st,
                       (const unsigned short*)dy, (const unsigned short*)x, b, (unsigned short*)dx, slab, T, I, R);
  } else if (nch <= 256) {
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<1>, dim3(blocks), dim3(256), 0, st, (const unsigned short*)dy,
                       (const unsigned short*)x, b, (unsigned short*)dx, slab, T, I);
  } else if (nch <= 512) {
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<2>, dim3(blocks), dim3(256), 0, st, (const unsigned short*)dy,
                       (const unsigned short*)x, b, (unsigned short*)dx, slab, T, I);
  } else if (nch <= 1024) {
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<4>, dim3(blocks), dim3(256), 0, st, (const unsigned short*)dy,
                       (const unsigned short*)x, b, (unsigned short*)dx, slab, T, I);
  } else {
    return -1;
  }
  INA_CHECK_LAUNCH();
  return 0;
}

int mha_lp(int L) { return L <= 32 ? 32 : (L <= 64 ? 64 : (L <= 96 ? 96 : (L <= 128 ? 128 : -1))); }

int mha_fwd(const BertMhaArgs& a, hipStream_t st) {
  const dim3 grid(a.S * a.nh);
  // 4 waves per (sequence, head) block: the forward is HBM-bound (q/k/v in, ctx out); 8 waves measured the
  // same (149 vs 151 us per layer, profiles/r5_mha/bert_sum_fwd8.txt)
#define CALL(LP)                                                                                          \
  hipLaunchKernelGGL((mha_fwd_kernel<LP, 4>), grid, dim3(256), 0, st, (const unsigned short*)a.qkv, a.inst, \
                     a.mask, a.S, a.L, a.nh, (unsigned short*)a.ctx, a.lse, a.salt, a.thr, a.inv_kp, a.drop)
  switch (mha_lp(a.L)) {
    case 32: CALL(32); break;
    case 64: CALL(64); break;
    case 96: CALL(96); break;
    case 128: CALL(128); break;
    default: return -1;
  }
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

int mha_bwd(const BertMhaArgs& a, hipStream_t st) {
  const dim3 grid(a.S * a.nh);
  // 8 waves per (sequence, head) block: one key / query tile per wave at L = 128, 16 waves per CU at the two
  // blocks the LDS allows (4 waves: 453 vs 379 us per layer, profiles/r5_mha/bert_sum_bwd4.txt / _bwd8.txt)
#define CALL(LP)                                                                                              \
  hipLaunchKernelGGL((mha_bwd_kernel<LP, 8>), grid, dim3(512), 0, st, (const unsigned short*)a.qkv,          \
                     (const unsigned short*)a.ctx, (const unsigned short*)a.dctx, a.lse, a.inst, a.mask, a.S, \
                     a.L, a.nh, (unsigned short*)a.dqkv, a.salt, a.thr, a.inv_kp, a.drop, a.bsum)
  switch (mha_lp(a.L)) {
    case 32: CALL(32); break;
    case 64: CALL(64); break;
    case 96: CALL(96); break;
    case 128: CALL(128); break;
    default: return -1;
  }
#undef CALL
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
