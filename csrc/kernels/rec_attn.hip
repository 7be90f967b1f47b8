// Word-level self-attention pooling straight from the BiLSTM step records, forward and backward
// (K4 of SURVEY 2.3; the bf16 training / eval path).
//
// Reference (model/layer_module.py:49-98, model/graph.py:36-53):
//   H      = DropoutWrapper output of the BiLSTM, [S, L, 2u]
//   x_proj = tanh(H @ W1 + b1);  score = x_proj @ w2;  alphas = softmax_t(score + (1 - (mask>0)) * -2^31)
//   e      = sum_t alphas_t H_t
//
// lstm_fwd leaves H in its step records [tile][dir][t][2 slots][U/4][64] (16-bit): h slot element
// [m][l] = unit 4m + (l >> 4) of sequence 16 tile + (l & 15).  hnat_attn / attn_bwd3 first
// transposed these into natural rows [S][L][2u] (a 300 MB round trip per 2048 episodes plus a
// bank-conflicted LDS scatter).  These kernels never transpose H: one wave owns a 16-sequence tile
// and walks its tokens, with the SEQUENCES on the MFMA columns:
//   * lane (q, n) holds, per token, the features F_q = {d u + 4m + q : d < 2, m < u/4} of sequence
//     n -- exactly its own record elements (one coalesced 128-B row per (dir, m) and step);
//   * the projection P^T[j][seq] = W1^T[j][k] H^T[k][seq] contracts over k in that lane-permuted
//     order (the A fragments, w1r, are packed to match: ops/packing.py::_attn_rec_idx), so the B
//     operand is the lane's own values; the accumulator rows j = 16 mt + 4 q + r land per lane;
//   * score / softmax / pooling are per column: a 4-group cross-lane sum gives every lane its
//     sequence's score, and an online (running-max) softmax pools e in registers in one pass;
//   * backward: dH^T = W1 dP^T feeds the dP accumulator straight back as the B operand (K = j in
//     accumulator order; w1rt packed to match) and its rows come out as each lane's own features,
//     i.e. dH leaves in the step-record lane layout that lstm_bwd reads with coalesced loads.
//     dW1 = sum H^T dP contracts over the sequences: both operands are staged per step pair in
//     lane-permuted [32 samples][columns] LDS images (4-/8-B stores) and read back transposed by
//     ds_read_b64_tr_b16 for v_mfma_f32_16x16x32_bf16 (K = 32 samples).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;


namespace {

template <int U>
struct RA {
  static constexpr int U4 = U / 4, H2 = 2 * U;
  static constexpr int NV = 2 * U4;                         // features per lane (both directions)
  static constexpr int NKR = (NV + 7) / 8;                  // projection K-steps (8 slots per lane)
  static constexpr int MT = (H2 + 15) / 16;                 // projection row tiles (j)
  static constexpr int NJ = 4 * MT;                         // dP values per lane
  static constexpr int NKS2 = (NJ + 7) / 8;                 // dH K-steps
  static constexpr int NRT = (NV + 3) / 4;                  // dH row tiles
  static constexpr int NVP = (NV + 1) & ~1;                 // H image columns per lane group (even)
  static constexpr int HT = (4 * NVP + 15) / 16;            // dW1 row tiles (H image columns)
  static constexpr int DEP = (NV + 3) & ~3;                 // de floats per lane in LDS (16-B reads)
  static constexpr int HCP = HT * 16 + 4, JCP = MT * 16 + 4;   // image row strides (elements)
  static constexpr int NA = MT * NKR * 64, NA2 = NRT * NKS2 * 64;
  static constexpr int RSTEP = 2 * U4 * 64;                 // record elements per (dir, step)
  static constexpr int WAVE_IMG = 32 * (HCP + JCP) * 2 + 64 * DEP * 4;   // bytes per wave (images | de)
  static constexpr int NS = H2 * H2 + 2 * H2;               // slab floats
  static_assert(U % 4 == 0 && NV <= 16, "rec_attn: u must be a multiple of 4, <= 32");
};

// feature index of slot idx (< NV) of lane group q
template <int U>
INA_DEVICE int rfeat(int idx, int q) {
  constexpr int U4 = U / 4;
  return (idx / U4) * U + 4 * (idx % U4) + q;
}

INA_DEVICE uint32_t cross_group_or(uint32_t v) {
  float a, b;
  dpp::swap16(__builtin_bit_cast(float, v), a, b);
  v = __builtin_bit_cast(uint32_t, a) | __builtin_bit_cast(uint32_t, b);
  dpp::swap32(__builtin_bit_cast(float, v), a, b);
  return __builtin_bit_cast(uint32_t, a) | __builtin_bit_cast(uint32_t, b);
}

// one step of the tile's records: the lane's NV h values (16-bit) and its two keep bytes
template <int U>
struct RecStep {
  unsigned short h[RA<U>::NV];
  uint32_t k0, k1;   // raw keep bytes of the two directions
  uint32_t kb;             // combined keep bits (set by rec_pin in the consuming step)
  float al;                // backward: alpha of the step (prefetched with the records)
};
// k0 / k1 always point at readable memory (the records themselves without dropout) and kor = 0xFFFF
// then sets every keep bit: no branch around the loads (an exec-masked load block here made the
// compiler wait vmcnt(0) right after issuing the prefetch)
template <int U>
INA_DEVICE void rec_load(const unsigned short* r0, const unsigned short* r1, const unsigned char* k0,
                         const unsigned char* k1, uint32_t kor, int t, RecStep<U>& o) {
  constexpr int U4 = RA<U>::U4, RSTEP = RA<U>::RSTEP;
#pragma unroll
  for (int m = 0; m < U4; ++m) {
    o.h[m] = r0[t * RSTEP + m * 64];
    o.h[U4 + m] = r1[t * RSTEP + m * 64];
  }
  o.k0 = k0[t * 64];
  o.k1 = k1[t * 64];
}
// first thing in the consuming step: pins the raw load results there and only then combines the keep
// bytes.  Any arithmetic on a prefetched value (the keep-byte combine at the load, or a pure op the
// scheduler hoists) forces vmcnt(0) right after the prefetch is issued, i.e. no overlap at all.
template <int U, bool AL>
INA_DEVICE void rec_pin(RecStep<U>& s, uint32_t kor) {
#pragma unroll
  for (int i = 0; i < RA<U>::NV; ++i) asm volatile("" : "+v"(s.h[i]));
  asm volatile("" : "+v"(s.k0));
  asm volatile("" : "+v"(s.k1));
  if constexpr (AL) asm volatile("" : "+v"(s.al));
  s.kb = ((uint32_t)s.k0 | ((uint32_t)s.k1 << 8)) | kor;
}
// token loop over ping-pong step buffers (2x unrolled): the prefetch of step t+1 goes into the other
// buffer, so no register copy of in-flight load results (a cur = nxt rotation forces vmcnt(0) at
// the loop latch, i.e. no overlap at all)
#ifndef INA_RA_PF_FWD
#define INA_RA_PF_FWD 1   // forward prefetch distance in token steps (1: two buffers, 2: three)
#endif
template <int U, int PF, class LD, class F>
INA_DEVICE void rec_steps(int L, LD&& load, F&& step) {
  if constexpr (PF == 1) {
  RecStep<U> a, b;
  load(0, a);
  int t = 0;
  for (; t + 1 < L; t += 2) {
    load(t + 1, b);
    step(t, a);
    load(t + 2 < L ? t + 2 : t + 1, a);
    step(t + 1, b);
  }
  if (t < L) step(t, a);
  } else {
  RecStep<U> a, b, c;
  auto cl = [&](int x) { return x < L ? x : L - 1; };
  load(0, a);
  load(cl(1), b);
  int t = 0;
  for (; t + 2 < L; t += 3) {
    load(t + 2, c);
    step(t, a);
    load(cl(t + 3), a);
    step(t + 1, b);
    load(cl(t + 4), b);
    step(t + 2, c);
  }
  if (t < L) step(t, a);
  if (t + 1 < L) step(t + 1, b);
  }
}
// DropoutWrapper output (model/graph.py:36-38): keep ? bf16(h / keep_prob) : 0 -- the same rounding
// as h_natural_kernel, so both attention paths see identical H.  Branch-free: the lane's keep bit of slot i as a
// 0 / all-ones mask (v_bfe_i32 of the 1-bit field) ANDed into the raw bf16 value (inv_kp = 1 and all bits set
// without dropout, which reproduces h exactly).  (Scaling by keep bit * inv_kp took an extract, a convert and a
// multiply per value.)  Two values per call: packed bf16 pair (B operand word) and the rounded fp32 values.
template <int U>
INA_DEVICE uint32_t rec_kmask(const RecStep<U>& s, int i) {
  constexpr int U4 = RA<U>::U4;
  const int b = i < U4 ? i : 8 + i - U4;
  return (uint32_t)__builtin_amdgcn_sbfe((int)s.kb, b, 1);
}
template <int U>
INA_DEVICE uint32_t rec_drop2(const RecStep<U>& s, int i, float inv_kp, float& v0, float& v1) {
  const float x0 = __builtin_bit_cast(float, ((uint32_t)s.h[i] & rec_kmask<U>(s, i)) << 16) * inv_kp;
  const float x1 = __builtin_bit_cast(float, ((uint32_t)s.h[i + 1] & rec_kmask<U>(s, i + 1)) << 16) * inv_kp;
  const uint32_t w = (uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16);
  v0 = __builtin_bit_cast(float, w << 16);
  v1 = __builtin_bit_cast(float, w & 0xFFFF0000u);
  return w;
}

INA_DEVICE u16x8_t tr8(const unsigned short* img, int stride, int c0, int q, int n) {
  const s16x4_t lo = tr_read(img + (8 * q + (n >> 2)) * stride + c0 + 4 * (n & 3));
  const s16x4_t hi = tr_read(img + (8 * q + 4 + (n >> 2)) * stride + c0 + 4 * (n & 3));
  return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                 (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
}

}  // namespace

// ------------------------------------------------------------------------------------------
// forward: one wave per tile, 4 tiles per workgroup.  Outputs e [S][2u] and alphas [S][L] (fp32).
// The raw scores are parked in LDS (lane q stores the steps t = q mod 4 and re-reads only its own
// stores) and normalised into alphas once the running max / sum are final.
// ------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(256) void rec_attn_fwd_kernel(
    const unsigned short* __restrict__ rec, const unsigned char* __restrict__ dmask, int S, int L, float inv_kp,
    const int* __restrict__ inst, const int* __restrict__ maskarr, const u16x8_t* __restrict__ w1r,
    const float* __restrict__ b1, const float* __restrict__ w2, float* __restrict__ e_out,
    float* __restrict__ alphas, const int* __restrict__ tlen, const int* __restrict__ perm) {
  using C = RA<U>;
  constexpr int U4 = C::U4, H2 = C::H2, NV = C::NV, NKR = C::NKR, MT = C::MT;
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15;
  // longest tiles first (the ragged plan sorts rows by length ascending; dispatching in that order left the longest
  // tiles for the kernel's tail): tile = ntiles - 1 - (4 blockIdx.x + wave)
  const int ntl = (S + 15) / 16, tix = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = ntl - 1 - tix;
  // weights shared by the workgroup in LDS (registers kept for occupancy: the loop is latency-bound
  // on the record loads, so resident waves are what hides them)
  __shared__ u16x8_t lA[MT * NKR * 64];
  __shared__ float lbw[2 * MT * 16];   // [b1 | w2]
  // raw scores [t][sequence] per wave (L <= 64): LDS, not alphas -- an exec-masked global store in
  // the step loop made the compiler drain vmcnt (the prefetch) at the join after it
  __shared__ float lsc[4][64 * 16];
  float* sl = lsc[threadIdx.x >> 6];
  for (int i = threadIdx.x; i < MT * NKR * 64; i += 256) lA[i] = w1r[i];
  for (int i = threadIdx.x; i < MT * 16; i += 256) {
    lbw[i] = i < H2 ? b1[i] : 0.f;
    lbw[MT * 16 + i] = i < H2 ? w2[i] : 0.f;
  }
  __syncthreads();
  if (tile < 0 || tile * 16 >= S) return;   // wave-uniform; no workgroup barrier after this point
  const int seq = tile * 16 + n;
  const bool valid = seq < S;
  const int seqc = valid ? seq : S - 1;
  // ragged tiles: the tile's steps t >= Lt are padding of every row (alpha exactly 0): not visited;
  // output rows go to perm[seq] (the records are in length-sorted row order)
  const int Lt = tlen ? tlen[tile] : L;
  const int orow = perm ? perm[seqc] : seqc;
  // token mask of the lane's sequence as a 64-bit set (L <= 64): 16 loads per lane, OR over the groups
  uint32_t mlo = 0, mhi = 0;
  {
    const int* mrow = maskarr + (long)inst[seqc] * L;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int t = q + 4 * i;
      const int v = mrow[t < L ? t : L - 1];
      const uint32_t on = (t < L && v > 0) ? 1u : 0u;
      if (i < 8) mlo |= on << t;
      else mhi |= on << (t - 32);
    }
    mlo = cross_group_or(mlo);
    mhi = cross_group_or(mhi);
  }
  const bool drop = dmask != nullptr;
  const unsigned short* r0 = rec + (size_t)tile * 2 * L * C::RSTEP + lane;
  const unsigned short* r1 = r0 + (size_t)L * C::RSTEP;
  const unsigned char* k0 = drop ? dmask + (size_t)tile * 2 * L * 64 + lane : reinterpret_cast<const unsigned char*>(r0);
  const unsigned char* k1 = drop ? k0 + (size_t)L * 64 : k0;
  const uint32_t kor = drop ? 0u : 0xFFFFu;
  float* arow = alphas + (size_t)orow * L;
  // sum_j w_j tanh(x_j) = sum_j w_j - 2 sum_j w_j r_j (tanh_r): the lane's share of sum_j w_j
  float wl = 0.f;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) wl += lbw[MT * 16 + 16 * m + 4 * q + r];
  float mx = -INFINITY, lsum = 0.f, ea[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) ea[i] = 0.f;
  auto load = [&](int t, RecStep<U>& o) { rec_load<U>(r0, r1, k0, k1, kor, t, o); };
  rec_steps<U, INA_RA_PF_FWD>(Lt, load, [&](int t, RecStep<U>& cur) {
    rec_pin<U, false>(cur, kor);
    float v[NV];
    u32x4_t Bw[NKR];
#pragma unroll
    for (int ks = 0; ks < NKR; ++ks) Bw[ks] = u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NV; i += 2) Bw[i / 8][(i % 8) / 2] = rec_drop2<U>(cur, i, inv_kp, v[i], v[i + 1]);
    u16x8_t B[NKR];
#pragma unroll
    for (int ks = 0; ks < NKR; ++ks) B[ks] = __builtin_bit_cast(u16x8_t, Bw[ks]);
    float sr = 0.f;
    asm volatile("" ::: "memory");   // re-read the LDS weights per step (no hoisting into registers)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const float4 bv = *reinterpret_cast<const float4*>(&lbw[16 * m + 4 * q]);
      const float4 wv = *reinterpret_cast<const float4*>(&lbw[MT * 16 + 16 * m + 4 * q]);
      f32x4_t acc = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int ks = 0; ks < NKR; ++ks) acc = mfma_bf16(lA[(m * NKR + ks) * 64 + lane], B[ks], acc);
      const f32x4_t rr = tanh_r4(acc);
      sr += wv.x * rr[0] + wv.y * rr[1] + wv.z * rr[2] + wv.w * rr[3];
    }
    const float sp = cross_group_sum(wl - 2.f * sr);
    const uint32_t on = t < 32 ? (mlo >> t) & 1u : (mhi >> (t - 32)) & 1u;
    const float sc = on ? sp : sp + -2147483648.f;
    // online softmax: rescale the running sum and pooled vector when the max moves
    const float mn = fmaxf(mx, sc);
    const float c = __expf(mx - mn), p = __expf(sc - mn);
    lsum = lsum * c + p;
#pragma unroll
    for (int i = 0; i < NV; ++i) ea[i] = ea[i] * c + p * v[i];
    mx = mn;
    if ((t & 3) == q) sl[t * 16 + n] = sc;
  });
  const float inv = 1.f / lsum;
  if (valid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) e_out[(size_t)orow * H2 + rfeat<U>(i, q)] = ea[i] * inv;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int t = q + 4 * i;
      if (t < L) arow[t] = t < Lt ? __expf(sl[t * 16 + n] - mx) * inv : 0.f;   // this lane's own LDS stores
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward: persistent grid, one wave per tile at a time, 4 waves per workgroup.  One pass over the
// tokens: sd = sum_t alpha_t d(alpha)_t = de . sum_t alpha_t H_t = de . e (the forward's output), so
// no separate d(alpha) pass; per step
//   recompute P, d(alpha)_t = de . H_t, ds_t = alpha_t (d(alpha)_t - sd), dP = ds w2 (1 - P^2),
//   dH_t = W1 dP_t + alpha_t de -> dHl [tiles][2][L][u/4][64] bf16 (lstm_bwd's lane layout), already
//   multiplied by the DropoutWrapper scale (keep bit * 1/keep_prob): the gradient w.r.t. the LSTM's
//   own output h, so lstm_bwd needs neither the keep bits nor a per-step mask,
//   dW1 += H^T dP (MFMAs per step pair), db1 += dP, dw2 += ds P (fp32: sum_t ds_t = 0 per sequence,
//   so these sums cancel heavily -- bf16 dP through the MFMA measured 1e-2 relative error on db1)
// slab per workgroup: [dW1 (H2*H2, row i, col j) | db1 (H2) | dw2 (H2)], the attn_bwd layout.
// ------------------------------------------------------------------------------------------
template <int U>
#ifndef INA_RA_PF_BWD
#define INA_RA_PF_BWD 2   // backward prefetch distance in token steps (1: two buffers, 2: three)
#endif
#ifndef INA_RA_BWD_WAVES
// 2 waves per SIMD with the 2-step prefetch (256 VGPRs, no spills): 5w5s 2,081,185 - 2,083,673 vs 2,064,695 -
// 2,072,628 episodes/s for 3 waves + 1 step (which spilled 18; 3 waves + 2 steps spills 270), profiles/r5_rapf
#define INA_RA_BWD_WAVES 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(U <= 20 ? INA_RA_BWD_WAVES : 2))) void rec_attn_bwd_kernel(
    const unsigned short* __restrict__ rec, const unsigned char* __restrict__ dmask, int S, int L, float inv_kp,
    const u16x8_t* __restrict__ w1r, const u16x8_t* __restrict__ w1rt, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ de, const float* __restrict__ e_fwd,
    const float* __restrict__ alphas, unsigned short* __restrict__ dHl, float* __restrict__ slab,
    const int* __restrict__ tlen, const int* __restrict__ perm) {
  using C = RA<U>;
  constexpr int U4 = C::U4, H2 = C::H2, NV = C::NV, NKR = C::NKR, MT = C::MT, NJ = C::NJ, NKS2 = C::NKS2,
                NRT = C::NRT, NVP = C::NVP, HT = C::HT, HCP = C::HCP, JCP = C::JCP, DEPC = C::DEP;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, n = lane & 15;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u16x8_t* lA = reinterpret_cast<u16x8_t*>(smem);
  u16x8_t* lAT = lA + C::NA;
  float* lbw = reinterpret_cast<float*>(lAT + C::NA2);   // [b1 | w2], MT * 16 each
  unsigned short* himg = reinterpret_cast<unsigned short*>(lbw + 2 * MT * 16) + (size_t)wave * (C::WAVE_IMG / 2);
  unsigned short* pimg = himg + 32 * HCP;
  for (int i = threadIdx.x; i < C::NA; i += 256) lA[i] = w1r[i];
  for (int i = threadIdx.x; i < C::NA2; i += 256) lAT[i] = w1rt[i];
  for (int i = threadIdx.x; i < MT * 16; i += 256) {
    lbw[i] = i < H2 ? b1[i] : 0.f;
    lbw[MT * 16 + i] = i < H2 ? w2[i] : 0.f;
  }
  float* lde = reinterpret_cast<float*>(pimg + 32 * JCP) + lane * C::DEP;   // the lane's de values
  // images zeroed once: pad columns (>= 4 NVP resp. 4 NJ) are never written and must read as 0
  for (int i = lane; i < C::WAVE_IMG / 4; i += 64) reinterpret_cast<uint32_t*>(himg)[i] = 0u;
  __syncthreads();

  f32x4_t accW[HT][MT];
#pragma unroll
  for (int a = 0; a < HT; ++a)
#pragma unroll
    for (int b = 0; b < MT; ++b) accW[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dw2a[MT][4], db1a[MT][4], sds = 0.f;   // dw2a: sum ds rr; sds: sum ds
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) dw2a[m][r] = db1a[m][r] = 0.f;
  const bool drop = dmask != nullptr;
  const int ntiles = (S + 15) / 16;

  // static round robin over the tiles in DESCENDING length (the plan sorts ascending): a wave's extra tile in the
  // last round is one of the shortest, not of the longest
  for (int ti = blockIdx.x * 4 + wave; ti < ntiles; ti += gridDim.x * 4) {   // wave-uniform
    const int tile = ntiles - 1 - ti;
    const int seq = tile * 16 + n;
    const bool valid = seq < S;
    const int seqc = valid ? seq : S - 1;
    const int Lt = tlen ? tlen[tile] : L;          // ragged tiles: dH rows t >= Lt are never read
    const int orow = perm ? perm[seqc] : seqc;     // de / e / alphas row of record row seq
    // de of the lane's features -> LDS (re-read per step: registers kept for occupancy)
    float sd = 0.f;
    lds_order();   // the previous tile's reads of lde come first
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const size_t o = (size_t)orow * H2 + rfeat<U>(i, q);
      const float x = valid ? de[o] : 0.f;
      lde[i] = x;
      sd = fmaf(x, e_fwd[o], sd);   // same sequential fma order as d(alpha) below: exact 0 for L = 1
    }
    sd = cross_group_sum(sd);
    const float* arow = alphas + (size_t)orow * L;
    const unsigned short* r0 = rec + (size_t)tile * 2 * L * C::RSTEP + lane;
    const unsigned short* r1 = r0 + (size_t)L * C::RSTEP;
    const unsigned char* k0 = drop ? dmask + (size_t)tile * 2 * L * 64 + lane : reinterpret_cast<const unsigned char*>(r0);
    const unsigned char* k1 = drop ? k0 + (size_t)L * 64 : k0;
    const uint32_t kor = drop ? 0u : 0xFFFFu;
    unsigned short* d0 = dHl + (size_t)tile * 2 * L * U4 * 64 + lane;   // dir 0; dir 1 at + L * U4 * 64
    auto load = [&](int t, RecStep<U>& o) {
      rec_load<U>(r0, r1, k0, k1, kor, t, o);
      o.al = arow[t];
    };
    rec_steps<U, INA_RA_PF_BWD>(Lt, load, [&](int t, RecStep<U>& cur) {
      rec_pin<U, true>(cur, kor);
      const float alv = valid ? cur.al : 0.f;
      float dev[DEPC];
      asm volatile("" ::: "memory");   // re-read de from LDS per step (no hoisting)
#pragma unroll
      for (int i = 0; i < DEPC; i += 4) {
        const float4 v4 = *reinterpret_cast<const float4*>(lde + i);
        dev[i] = v4.x; dev[i + 1] = v4.y; dev[i + 2] = v4.z; dev[i + 3] = v4.w;
      }
      // H (dropped, bf16 pairs) -> B operand and straight into the dW1 image (row 16 (t & 1) + n)
      const int rr = 16 * (t & 1) + n;
      uint32_t* hw = reinterpret_cast<uint32_t*>(himg + rr * HCP + q * NVP);
      u32x4_t Bw[NKR];
#pragma unroll
      for (int ks = 0; ks < NKR; ++ks) Bw[ks] = u32x4_t{0u, 0u, 0u, 0u};
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < NV; i += 2) {
        float v0, v1;
        const uint32_t w = rec_drop2<U>(cur, i, inv_kp, v0, v1);
        Bw[i / 8][(i % 8) / 2] = w;
        hw[i / 2] = w;
        d = fmaf(dev[i], v0, d);
        d = fmaf(dev[i + 1], v1, d);
      }
      u16x8_t B[NKR];
#pragma unroll
      for (int ks = 0; ks < NKR; ++ks) B[ks] = __builtin_bit_cast(u16x8_t, Bw[ks]);
      const float ds = alv * (cross_group_sum(d) - sd);   // 0 for padding sequences (alpha 0)
      const float ds4 = 4.f * ds;
      sds += ds;
      float dp[MT][4];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4_t acc;
        float wv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[r] = lbw[16 * m + 4 * q + r];
          wv[r] = lbw[MT * 16 + 16 * m + 4 * q + r];
        }
#pragma unroll
        for (int ks = 0; ks < NKR; ++ks) acc = mfma_bf16(lA[(m * NKR + ks) * 64 + lane], B[ks], acc);
        const f32x4_t r4 = tanh_r4(acc);                    // P = 1 - 2 rr, 1 - P^2 = 4 rr (1 - rr)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float rr = r4[r];
          dp[m][r] = ds4 * (wv[r] * (rr - rr * rr));
          dw2a[m][r] += ds * rr;                             // dw2 = sum ds P = sum ds - 2 sum ds rr
          db1a[m][r] += dp[m][r];
        }
      }
      // dH^T = W1 dP^T (+ alpha de): K = j in accumulator order, rows = the lane's own features
      u16x8_t B2[NKS2];
#pragma unroll
      for (int ks = 0; ks < NKS2; ++ks) {
        B2[ks] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int idx = ks * 8 + j;
          if (idx < NJ) B2[ks][j] = f2bf(dp[idx >> 2][idx & 3]);
        }
      }
#pragma unroll
      for (int T = 0; T < NRT; ++T) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS2; ++ks) acc = mfma_bf16(lAT[(T * NKS2 + ks) * 64 + lane], B2[ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int fi = 4 * T + r;
          if (fi < NV) {
            const int dd = fi / U4, m = fi % U4;
            d0[((size_t)dd * L + t) * U4 * 64 + m * 64] =
                (unsigned short)((uint32_t)f2bf((acc[r] + alv * dev[fi]) * inv_kp) & rec_kmask<U>(cur, fi));
          }
        }
      }
      // ---- stage dP for dW1 (image row rr), flush every step pair
#pragma unroll
      for (int m = 0; m < MT; ++m)
        *reinterpret_cast<u16x4_t*>(pimg + rr * JCP + q * NJ + 4 * m) =
            u16x4_t{f2bf(dp[m][0]), f2bf(dp[m][1]), f2bf(dp[m][2]), f2bf(dp[m][3])};
      if ((t & 1) || t == Lt - 1) {
        if (!(t & 1)) {
          // lone last step (L odd): rows 16..31 still hold the previous (already flushed) pair
#pragma unroll
          for (int m = 0; m < MT; ++m)
            *reinterpret_cast<u16x4_t*>(pimg + (16 + n) * JCP + q * NJ + 4 * m) = u16x4_t{0, 0, 0, 0};
        }
        lds_order();
        u16x8_t fb[MT];
#pragma unroll
        for (int b = 0; b < MT; ++b) fb[b] = tr8(pimg, JCP, 16 * b, q, n);
#pragma unroll
        for (int a = 0; a < HT; ++a) {
          const u16x8_t fa = tr8(himg, HCP, 16 * a, q, n);
#pragma unroll
          for (int b = 0; b < MT; ++b) accW[a][b] = mfma_bf16(fa, fb[b], accW[a][b]);
        }
        lds_order();   // the next pair's stores come after these reads (in-order LDS)
      }
    });
  }
  // ---- workgroup reduction into the slab (LDS reused as fp32 after a barrier)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  for (int i = threadIdx.x; i < C::NS; i += 256) red[i] = 0.f;
  __syncthreads();
  float d1s[MT][4], d2s[MT][4];   // cross-lane sums first (every lane takes part in the shuffles)
  const float sdsum = group16_sum(sds);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d1s[m][r] = group16_sum(db1a[m][r]);
      d2s[m][r] = sdsum - 2.f * group16_sum(dw2a[m][r]);
    }
  // un-permute the image columns: H column c -> feature i, dP column c' -> projection row j
  int jmap[MT];
#pragma unroll
  for (int b = 0; b < MT; ++b) {
    const int c = 16 * b + n, qq = c / NJ, idx = c % NJ;
    const int j = 16 * (idx >> 2) + 4 * qq + (idx & 3);
    jmap[b] = (qq < 4 && j < H2) ? j : -1;
  }
  ordered_wave_accumulate(wave, 4, [&] {   // deterministic summation order
#pragma unroll
    for (int a = 0; a < HT; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * a + 4 * q + r, qq = c / NVP, idx = c % NVP;
        if (qq >= 4 || idx >= NV) continue;
        const int row = rfeat<U>(idx, qq) * H2;
#pragma unroll
        for (int b = 0; b < MT; ++b)
          if (jmap[b] >= 0) red[row + jmap[b]] += accW[a][b][r];
      }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * m + 4 * q + r;
        if (n == 0 && j < H2) {
          red[H2 * H2 + j] += d1s[m][r];
          red[H2 * H2 + H2 + j] += d2s[m][r];
        }
      }
  });
  for (int i = threadIdx.x; i < C::NS; i += 256) slab[(size_t)blockIdx.x * C::NS + i] = red[i];
}

// ------------------------------------------------------------------------------------------
namespace ina {

template <int U>
static size_t rec_attn_bwd_lds() {
  using C = RA<U>;
  const size_t b = (size_t)(C::NA + C::NA2) * 16 + 2 * C::MT * 16 * 4 + 4 * (size_t)C::WAVE_IMG;
  const size_t r = (size_t)C::NS * 4;
  return b > r ? b : r;
}

template <int U>
static int rec_attn_fwd_t(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a,
                          hipStream_t st) {
  const int ntiles = (a.S + 15) / 16;
  hipLaunchKernelGGL((rec_attn_fwd_kernel<U>), dim3((ntiles + 3) / 4), dim3(256), 0, st, (const unsigned short*)rec,
                     dmask, a.S, a.L, inv_kp, a.inst, a.mask, (const u16x8_t*)a.w1pack, a.b1, a.w2, a.e, a.alphas,
                     a.tlen, a.perm);
  INA_CHECK_LAUNCH();
  return 0;
}

template <int U>
static int rec_attn_bwd_t(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a,
                          hipStream_t st) {
  const size_t lds = rec_attn_bwd_lds<U>();
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)rec_attn_bwd_kernel<U>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  hipLaunchKernelGGL((rec_attn_bwd_kernel<U>), dim3(a.blocks), dim3(256), lds, st, (const unsigned short*)rec, dmask,
                     a.S, a.L, inv_kp, (const u16x8_t*)a.w1pack, (const u16x8_t*)a.w1tpack, a.b1, a.w2, a.de,
                     a.e, a.alphas, (unsigned short*)a.dHraw, a.slab, a.tlen, a.perm);
  INA_CHECK_LAUNCH();
  return 0;
}

template <int U>
static int rec_attn_bwd_resident_t() {
  static int cached = -1;
  if (cached >= 0) return cached;
  const size_t lds = rec_attn_bwd_lds<U>();
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)rec_attn_bwd_kernel<U>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rec_attn_bwd_kernel<U>, 256, lds) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    per_cu = cus = 0;
  cached = per_cu * cus;
  return cached;
}

#define INA_RA_DISPATCH(EXPR_U) \
  if (U == 8) return EXPR_U(8); \
  if (U == 20) return EXPR_U(20); \
  if (U == 32) return EXPR_U(32); \
  return -1;

int rec_attn_fwd(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a, int U, hipStream_t st) {
  if (a.S <= 0) return 0;
#define INA_RA_F(UV) rec_attn_fwd_t<UV>(rec, dmask, inv_kp, a, st)
  INA_RA_DISPATCH(INA_RA_F)
#undef INA_RA_F
}
int rec_attn_bwd(const void* rec, const unsigned char* dmask, float inv_kp, const AttnArgs& a, int U, hipStream_t st) {
  if (a.S <= 0) return 0;
#define INA_RA_B(UV) rec_attn_bwd_t<UV>(rec, dmask, inv_kp, a, st)
  INA_RA_DISPATCH(INA_RA_B)
#undef INA_RA_B
}
int rec_attn_bwd_resident_blocks(int U) {
#define INA_RA_R(UV) rec_attn_bwd_resident_t<UV>()
  INA_RA_DISPATCH(INA_RA_R)
#undef INA_RA_R
}
#undef INA_RA_DISPATCH

}  // namespace ina
