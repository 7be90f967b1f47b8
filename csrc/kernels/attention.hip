// Fused word-level self-attention pooling, forward and backward (K4 of SURVEY 2.3).
//
// Reference (model/layer_module.py:49-98, model/graph.py:52-53):
//   x_proj = tanh(H @ W1 + b1)            W1 = self_attn/dense/kernel [2u, 2u]
//   score  = x_proj @ W_a2                W_a2 [2u, 1]
//   alphas = softmax_t(score + (1 - (mask>0)) * -2^31)
//   e      = sum_t alphas_t * H_t
// H is the BiLSTM output *after* the DropoutWrapper output dropout, applied once by lstm_fwd
// (which stores the dropped copy); lstm_bwd re-applies the mask to the dH this kernel returns.
//
// One wave processes one sentence at a time (grid-stride).  The projection is computed
// transposed, P^T[j, tok] = W1^T[j, i] H^T[i, tok], with v_mfma_f32_16x16x32_bf16 (or the f32
// 16x16x4 form): the B operand is 8 contiguous features of one token (one 16-B load), and the
// accumulator puts the sentence's tokens on the lane columns so the score / softmax / pooling
// reductions are 16-lane shuffles.  Backward recomputes P, forms dP^T in the accumulator
// layout and feeds it straight back as the B operand of dH^T = W1 dP^T; dW1 = H^T dP is
// accumulated with MFMAs after a wave-private LDS transpose (tokens become the K dimension).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

template <bool BF16>
struct FT;
template <>
struct FT<true> {
  using frag = u16x8_t;
  using elem = unsigned short;
  static constexpr int KPL = 8;
};
template <>
struct FT<false> {
  using frag = float;
  using elem = float;
  static constexpr int KPL = 1;
};

INA_DEVICE f32x4_t mma(const u16x8_t& a, const u16x8_t& b, const f32x4_t& c) { return mfma_bf16(a, b, c); }
INA_DEVICE f32x4_t mma(float a, float b, const f32x4_t& c) { return mfma_f32(a, b, c); }
INA_DEVICE void fset(u16x8_t& f, int j, float v) { f[j] = f2bf(v); }
INA_DEVICE void fset(float& f, int, float v) { f = v; }
INA_DEVICE float ld_elem(const unsigned short* p) { return bf2f(*p); }
INA_DEVICE float ld_elem(const float* p) { return *p; }
INA_DEVICE unsigned short cvt_elem(float v, unsigned short*) { return f2bf(v); }
INA_DEVICE float cvt_elem(float v, float*) { return v; }
INA_DEVICE float rnd(float v, bool bf16) { return bf16 ? round_bf(v) : v; }

INA_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int U, int NT, bool BF16>
struct AShape {
  static constexpr int H2 = 2 * U;
  static constexpr int KPL = FT<BF16>::KPL;
  static constexpr int KP = BF16 ? ((H2 + 31) / 32) * 32 : ((H2 + 3) / 4) * 4;  // padded feature dim
  static constexpr int NKS = BF16 ? KP / 32 : KP / 4;                           // proj K-steps
  static constexpr int MT = (H2 + 15) / 16;                                      // j tiles
  static constexpr int NKS2 = (4 * MT + KPL - 1) / KPL;                          // dH K-steps (j slots)
  static constexpr int NV = BF16 ? NKS * 8 : NKS;                               // features per lane per token
  static constexpr int TOKP = ((NT * 16 + 31) / 32) * 32;                        // LDS token columns
  static constexpr int RS = TOKP + (BF16 ? 8 : 4);                              // LDS row stride (elements)
};

// feature index held in slot v (0..NV-1) of lane group q
template <bool BF16>
INA_DEVICE int feat_of(int v, int q) {
  if (BF16) return (v >> 3) * 32 + 8 * q + (v & 7);
  return 4 * v + q;
}

// Load the (already dropout-applied, by lstm_fwd) H values of token `tok` for lane group q.  Every
// load is unconditional (clamped address + select): a lane-dependent branch around a load makes
// hipcc wait vmcnt(0) per element and serialises the L2 round trips.
template <int U, int NT, bool BF16>
INA_DEVICE void load_h(const typename FT<BF16>::elem* hraw, long seq, int tok, int L, int q, float* hv) {
  using Sh = AShape<U, NT, BF16>;
  constexpr int H2 = Sh::H2;
  const bool tv = tok < L;
  const long row = (seq * L + (tv ? tok : L - 1)) * H2;
  if constexpr (BF16) {
#pragma unroll
    for (int ks = 0; ks < Sh::NKS; ++ks) {
      const int k0 = 32 * ks + 8 * q;
      const bool ok = tv && (k0 < H2);
      const u16x8_t v = *reinterpret_cast<const u16x8_t*>(hraw + row + (ok ? k0 : 0));
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) hv[ks * 8 + jj] = ok ? bf2f(v[jj]) : 0.f;
    }
  } else {
#pragma unroll
    for (int v = 0; v < Sh::NV; ++v) {
      const int k = feat_of<BF16>(v, q);
      const bool ok = tv && (k < H2);
      const float x = ld_elem(hraw + row + (ok ? k : 0));
      hv[v] = ok ? x : 0.f;
    }
  }
}

// bf16 forward of one sentence from its H tiles (hf: token 16 * nt + n, features 32 * ks + 8 * q ..+7,
// zero outside [L) x [2U)) and the mask ids of those tokens: projection (MFMA), tanh, w2 dot, masked
// softmax over the tokens, pooling.  Weight operands read through wa / wb / ww (register arrays).
template <int MT, int NKS>
struct RegW {
  const u16x8_t (&A)[MT][NKS];
  const float (&bj)[MT][4];
  const float (&wj)[MT][4];
  INA_DEVICE u16x8_t wa(int m, int ks) const { return A[m][ks]; }
  INA_DEVICE float wb(int m, int r) const { return bj[m][r]; }
  INA_DEVICE float ww(int m, int r) const { return wj[m][r]; }
};

template <int U, int NT, typename W>
INA_DEVICE void attn_sentence_bf16(const u16x8_t (&hf)[NT][AShape<U, NT, true>::NKS], const int (&mk)[NT],
                                   const W& w, long s, int L, int q, int n,
                                   float* __restrict__ e_out, float* __restrict__ alphas) {
  using Sh = AShape<U, NT, true>;
  constexpr int H2 = Sh::H2, NKS = Sh::NKS, MT = Sh::MT;
  float score[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int tok = 16 * nt + n;
    float sp = 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      f32x4_t acc = {w.wb(m, 0), w.wb(m, 1), w.wb(m, 2), w.wb(m, 3)};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) acc = mma(w.wa(m, ks), hf[nt][ks], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) sp += w.ww(m, r) * tanhf_(acc[r]);
    }
    sp = cross_group_sum(sp);
    const float m01 = mk[nt] > 0 ? 1.f : 0.f;
    score[nt] = (tok < L) ? sp + (1.f - m01) * -2147483648.f : -INFINITY;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) mx = fmaxf(mx, score[nt]);
  mx = group16_max(mx);
  float p[NT], sum = 0.f;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    p[nt] = (16 * nt + n < L) ? __expf(score[nt] - mx) : 0.f;
    sum += p[nt];
  }
  sum = group16_sum(sum);
  const float inv = 1.f / sum;
  float ev[NKS][8];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) ev[ks][j] = 0.f;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int tok = 16 * nt + n;
    const float a = p[nt] * inv;
    if (q == 0 && tok < L) alphas[(long)s * L + tok] = a;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) ev[ks][j] += a * bf2f(hf[nt][ks][j]);
  }
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) ev[ks][j] = group16_sum(ev[ks][j]);
  if (n == 0) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int k0 = 32 * ks + 8 * q;
      if (k0 < H2) {
        float4* o = reinterpret_cast<float4*>(e_out + (long)s * H2 + k0);
        o[0] = make_float4(ev[ks][0], ev[ks][1], ev[ks][2], ev[ks][3]);
        o[1] = make_float4(ev[ks][4], ev[ks][5], ev[ks][6], ev[ks][7]);
      }
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------
template <int U, int NT, bool BF16>
__global__ __launch_bounds__(256) void attn_fwd_kernel(
    const typename FT<BF16>::elem* hraw, const int* __restrict__ inst, const int* __restrict__ maskarr,
    int S, int L, const typename FT<BF16>::frag* __restrict__ w1pack, const float* __restrict__ b1,
    const float* __restrict__ w2, float* __restrict__ e_out,
    float* __restrict__ alphas) {
  using Sh = AShape<U, NT, BF16>;
  using frag = typename FT<BF16>::frag;
  constexpr int H2 = Sh::H2, NKS = Sh::NKS, MT = Sh::MT, NV = Sh::NV, KPL = Sh::KPL;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, n = lane & 15;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  frag A[MT][NKS];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) A[m][ks] = w1pack[(m * NKS + ks) * 64 + lane];
  float bj[MT][4], wj[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * m + 4 * q + r;
      bj[m][r] = j < H2 ? b1[j] : 0.f;
      wj[m][r] = j < H2 ? w2[j] : 0.f;
    }
  for (int s = gw; s < S; s += nw) {
    const long row = (long)inst[s] * L;
    if constexpr (BF16) {
      // all of the sentence's loads first (H tiles stay in registers for scores AND pooling)
      u16x8_t hf[NT][NKS];
      int mk[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int tok = 16 * nt + n;
        const bool tv = tok < L;
        const size_t hrow = ((size_t)s * L + (tv ? tok : L - 1)) * H2;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const int k0 = 32 * ks + 8 * q;
          const bool ok = tv && (k0 < H2);
          const u16x8_t v = *reinterpret_cast<const u16x8_t*>(hraw + hrow + (ok ? k0 : 0));
          hf[nt][ks] = ok ? v : u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        }
        mk[nt] = maskarr[row + (tv ? tok : L - 1)];
      }
      attn_sentence_bf16<U, NT>(hf, mk, RegW<MT, NKS>{A, bj, wj}, s, L, q, n, e_out, alphas);
      continue;
    }
    // pass 1: scores (projection + tanh + w2 dot), one token tile at a time
    float score[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tok = 16 * nt + n;
      float hv[NV];
      load_h<U, NT, BF16>(hraw, s, tok, L, q, hv);
      frag B[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
        for (int j = 0; j < KPL; ++j) fset(B[ks], j, rnd(hv[ks * KPL + j], BF16));
      }
      float sp = 0.f;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4_t acc = {bj[m][0], bj[m][1], bj[m][2], bj[m][3]};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) acc = mma(A[m][ks], B[ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) sp += wj[m][r] * tanhf_(acc[r]);
      }
      sp = cross_group_sum(sp);
      const int mk = maskarr[row + (tok < L ? tok : L - 1)];
      const float m01 = mk > 0 ? 1.f : 0.f;
      score[nt] = (tok < L) ? sp + (1.f - m01) * -2147483648.f : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) mx = fmaxf(mx, score[nt]);
    mx = group16_max(mx);
    float p[NT], sum = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      p[nt] = (16 * nt + n < L) ? __expf(score[nt] - mx) : 0.f;
      sum += p[nt];
    }
    sum = group16_sum(sum);
    const float inv = 1.f / sum;
    asm volatile("" ::: "memory");  // keep pass-2 loads as re-reads (no CSE across passes)
    // pass 2: pooling (H re-read from L1/L2)
    float ev[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) ev[v] = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tok = 16 * nt + n;
      const float a = p[nt] * inv;
      if (q == 0 && tok < L) alphas[(long)s * L + tok] = a;
      float hv[NV];
      load_h<U, NT, BF16>(hraw, s, tok, L, q, hv);
#pragma unroll
      for (int v = 0; v < NV; ++v) ev[v] += a * hv[v];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) ev[v] = group16_sum(ev[v]);
    if (n == 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = feat_of<BF16>(v, q);
        if (k < H2) e_out[(long)s * H2 + k] = ev[v];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// slab per block: [dW1 (H2*H2, row i, col j) | db1 (H2) | dw2 (H2)]
template <int U, int NT, bool BF16>
__global__ __launch_bounds__(256) void attn_bwd_kernel(
    const typename FT<BF16>::elem* hraw, const int* __restrict__ inst, int S, int L,
    const typename FT<BF16>::frag* __restrict__ w1pack, const typename FT<BF16>::frag* __restrict__ w1tpack,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ de,
    const float* __restrict__ alphas, typename FT<BF16>::elem* __restrict__ dHraw,
    float* __restrict__ slab) {
  using Sh = AShape<U, NT, BF16>;
  using frag = typename FT<BF16>::frag;
  using elem = typename FT<BF16>::elem;
  constexpr int H2 = Sh::H2, NKS = Sh::NKS, MT = Sh::MT, NV = Sh::NV, KPL = Sh::KPL, NKS2 = Sh::NKS2,
                TOKP = Sh::TOKP, RS = Sh::RS;
  constexpr int ROWS = MT * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, n = lane & 15;
  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  elem* HT = reinterpret_cast<elem*>(smem) + (size_t)wave * 2 * ROWS * RS;  // [i][tok]
  elem* DPT = HT + ROWS * RS;                                                  // [j][tok]
  for (int i = lane; i < 2 * ROWS * RS; i += 64) HT[i] = cvt_elem(0.f, (elem*)nullptr);
  wave_lds_sync();

  float bj[MT][4], wj[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * m + 4 * q + r;
      bj[m][r] = j < H2 ? b1[j] : 0.f;
      wj[m][r] = j < H2 ? w2[j] : 0.f;
    }
  f32x4_t accW[MT][MT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < MT; ++b) accW[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dw2a[MT][4], db1a[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) dw2a[m][r] = db1a[m][r] = 0.f;

  for (int s = gw; s < S; s += nw) {
    // de for the lane's features
    float dev[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int k = feat_of<BF16>(v, q);
      const float x = de[(long)s * H2 + (k < H2 ? k : 0)];
      dev[v] = k < H2 ? x : 0.f;
    }
    float dei[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * m + 4 * q + r;
        const float x = de[(long)s * H2 + (i < H2 ? i : 0)];
        dei[m][r] = i < H2 ? x : 0.f;
      }
    // pass 1: d(alpha)_t = de . H_t and the softmax-backward dot sum_t alpha_t d(alpha)_t
    float al[NT], da[NT];
#pragma unroll 1
    for (int nt = 0; nt < NT; ++nt) {
      const int tok = 16 * nt + n;
      float hv[NV];
      load_h<U, NT, BF16>(hraw, s, tok, L, q, hv);
      const float av = alphas[(long)s * L + (tok < L ? tok : L - 1)];
      float d = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) d += dev[v] * hv[v];
      d = cross_group_sum(d);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        if (j == nt) {  // compile-time register index (no scratch)
          al[j] = tok < L ? av : 0.f;
          da[j] = d;
        }
    }
    float sd = 0.f;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) sd += al[nt] * da[nt];
    sd = group16_sum(sd);
    asm volatile("" ::: "memory");  // keep pass-2 loads as re-reads (no CSE across passes)
    // pass 2: recompute the projection per token tile, form dP, dH, and stage dW1 operands
#pragma unroll 1
    for (int nt = 0; nt < NT; ++nt) {
      const int tok = 16 * nt + n;
      float alv = al[0], dav = da[0];
#pragma unroll
      for (int j = 1; j < NT; ++j)
        if (j == nt) {
          alv = al[j];
          dav = da[j];
        }
      float hv[NV];
      load_h<U, NT, BF16>(hraw, s, tok, L, q, hv);
      frag B[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
        for (int j = 0; j < KPL; ++j) fset(B[ks], j, rnd(hv[ks * KPL + j], BF16));
      }
      const float ds = alv * (dav - sd);
      float dp[MT][4];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4_t acc = {bj[m][0], bj[m][1], bj[m][2], bj[m][3]};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) acc = mma(w1pack[(m * NKS + ks) * 64 + lane], B[ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = tanhf_(acc[r]);
          dp[m][r] = ds * wj[m][r] * (1.f - pr * pr);
          dw2a[m][r] += ds * pr;
          db1a[m][r] += dp[m][r];
        }
      }
      // dH^T = W1 dP^T  (+ alpha * de), dropout mask re-applied
      frag B2[NKS2];
#pragma unroll
      for (int ks = 0; ks < NKS2; ++ks) {
        if constexpr (BF16) {
          B2[ks] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        } else {
          B2[ks] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
          const int idx = ks * KPL + j;
          if (idx < 4 * MT) fset(B2[ks], j, dp[idx >> 2][idx & 3]);
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS2; ++ks) acc = mma(w1tpack[(m * NKS2 + ks) * 64 + lane], B2[ks], acc);
        if (tok < L && 16 * m + 4 * q < H2) {
          f32x4_t g;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * m + 4 * q + r;
            (void)i;
            g[r] = acc[r] + alv * dei[m][r];
          }
          elem* dst = dHraw + ((long)s * L + tok) * H2 + 16 * m + 4 * q;
          if constexpr (BF16) {  // bf16 dH: halves the largest backward stream (read back by lstm_bwd)
            uint2 pk;
            pk.x = (uint32_t)f2bf(g[0]) | ((uint32_t)f2bf(g[1]) << 16);
            pk.y = (uint32_t)f2bf(g[2]) | ((uint32_t)f2bf(g[3]) << 16);
            *reinterpret_cast<uint2*>(dst) = pk;
          } else {
            *reinterpret_cast<f32x4_t*>(dst) = g;
          }
        }
      }
      // stage H (MFMA operand values) and dP for the dW1 MFMA; tokens are the K dimension
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = feat_of<BF16>(v, q);
        if (k < ROWS) HT[k * RS + tok] = cvt_elem(hv[v], (elem*)nullptr);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) DPT[(16 * m + 4 * q + r) * RS + tok] = cvt_elem(dp[m][r], (elem*)nullptr);
    }
    wave_lds_sync();
    if constexpr (BF16) {
#pragma unroll
      for (int kt = 0; kt < TOKP / 32; ++kt)
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          const u16x8_t fa = *reinterpret_cast<const u16x8_t*>(&HT[(16 * a + n) * RS + 32 * kt + 8 * q]);
#pragma unroll
          for (int b = 0; b < MT; ++b) {
            const u16x8_t fb = *reinterpret_cast<const u16x8_t*>(&DPT[(16 * b + n) * RS + 32 * kt + 8 * q]);
            accW[a][b] = mfma_bf16(fa, fb, accW[a][b]);
          }
        }
    } else {
#pragma unroll
      for (int kt = 0; kt < TOKP / 4; ++kt)
#pragma unroll
        for (int a = 0; a < MT; ++a) {
          const float fa = HT[(16 * a + n) * RS + 4 * kt + q];
#pragma unroll
          for (int b = 0; b < MT; ++b) {
            const float fb = DPT[(16 * b + n) * RS + 4 * kt + q];
            accW[a][b] = mfma_f32(fa, fb, accW[a][b]);
          }
        }
    }
    wave_lds_sync();
  }
  // ---- block reduction into the slab
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  const int NS = H2 * H2 + 2 * H2;
  for (int i = threadIdx.x; i < NS; i += 256) red[i] = 0.f;
  __syncthreads();
  float d1s[MT][4], d2s[MT][4];   // cross-lane sums first (every lane takes part in the shuffles)
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d1s[m][r] = group16_sum(db1a[m][r]);
      d2s[m][r] = group16_sum(dw2a[m][r]);
    }
  ordered_wave_accumulate(threadIdx.x >> 6, 4, [&] {   // 256-thread workgroups; deterministic order
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * a + 4 * q + r, j = 16 * b + n;
          if (i < H2 && j < H2) red[i * H2 + j] += accW[a][b][r];
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
  for (int i = threadIdx.x; i < NS; i += 256) slab[(size_t)blockIdx.x * NS + i] = red[i];
}

// ------------------------------------------------------------------------------------------
// bf16 backward, v3 (4-wave workgroups, one sentence per wave at a time, persistent grid):
//  * the NEXT sentence's H rows / alphas / de land in a wave-private LDS buffer by LDS-DMA
//    (global_load_lds) while the current one is processed: the HBM latency of the per-sentence
//    loads is off the critical path (v2 issued them at the top of each sentence: ~70 us of 317);
//  * dW1 = sum_t H_t^T dP_t per 16-token tile with v_mfma_f32_16x16x16_bf16, both operands read by
//    ds_read_b64_tr_b16 (hardware transpose): the A operand straight from the prefetched natural
//    H image, the B operand from a [16 tokens][ROWS] dP image written with 8-B stores (v2 staged
//    both through per-element 16-bit LDS stores: 84 ds_write_b16 per sentence);
//  * weight fragments shared by the block in LDS, as before.
// slab per block: [dW1 (H2*H2, row i, col j) | db1 (H2) | dw2 (H2)]
// ------------------------------------------------------------------------------------------
constexpr int AB3_WAVES = 4;

template <int U, int NT>
struct AB3 {
  static constexpr int H2 = 2 * U, MT = (H2 + 15) / 16, ROWS = MT * 16;
  static constexpr int NKS = (H2 + 31) / 32, NKS2 = (4 * MT + 7) / 8;
  static constexpr int TOK = NT * 16;                                  // image rows (tokens, zero padded)
  static constexpr int DEP = (32 * NKS > ROWS ? 32 * NKS : ROWS);      // de floats (zero padded)
  static constexpr int HIMG = TOK * H2 * 2;                            // bytes, bf16 [TOK][H2]
  static constexpr int BUF = HIMG + TOK * 4 + DEP * 4;                 // H image | alphas | de
  static constexpr int DPI = 16 * ROWS * 2;                            // bf16 dP image [16][ROWS]
  static constexpr int WAVE = 2 * BUF + DPI;
  static constexpr int NA = MT * NKS * 64, NA2 = MT * NKS2 * 64;
  static constexpr int HEAD = ((NA + NA2) * 16 + 2 * ROWS * 4 + 15) / 16 * 16;
  static_assert(HIMG % 16 == 0 && BUF % 16 == 0 && WAVE % 16 == 0, "16-B LDS carve");
};

// LDS-DMA (global_load_lds: each active lane's 16 / 4 bytes land at M0 + lane * size) issued by
// inline asm: through the builtin, LLVM's waitcnt pass assumes the in-flight DMA may alias every
// later LDS access of the kernel and waits vmcnt(0) before them, serialising the prefetch.  The
// kernel synchronises explicitly instead (s_waitcnt vmcnt(0) at the top of each sentence), and no
// other code in it uses M0.  An asm VMEM op unknown to the compiler can only make the compiler's
// own vmcnt waits longer, never shorter (in-order retirement), so its loads stay correct.
INA_DEVICE uint32_t lds_off(const void* p) {   // generic pointer into LDS -> 32-bit LDS address (M0)
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
INA_DEVICE void lds_dma16(const void* g, const void* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(m0) : "memory");
}
INA_DEVICE void lds_dma4(const void* g, const void* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds_wave_base));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(m0) : "memory");
}
// fp32 values of the prefetch buffer read through 16-bit vector types: with float-typed reads LLVM
// treats them as possibly aliasing the in-flight LDS-DMA into the other buffer and inserts a full
// vmcnt(0) wait before them (the prefetch latency back on the critical path)
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
INA_DEVICE float ldsf(const float* p) {
  const u16x2_t v = *reinterpret_cast<const u16x2_t*>(p);
  return __builtin_bit_cast(float, (uint32_t)v[0] | ((uint32_t)v[1] << 16));
}
INA_DEVICE void ldsf4(const float* p, float* o) {
  const u16x8_t v = *reinterpret_cast<const u16x8_t*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = __builtin_bit_cast(float, (uint32_t)v[2 * i] | ((uint32_t)v[2 * i + 1] << 16));
}
// (lds_order: also keeps the compiler from waiting on the in-flight prefetch DMA)

template <int U, int NT>
__global__ __launch_bounds__(256) void attn_bwd3_kernel(
    const unsigned short* __restrict__ hraw, int S, int L, const u16x8_t* __restrict__ w1pack,
    const u16x8_t* __restrict__ w1tpack, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ de, const float* __restrict__ alphas, unsigned short* __restrict__ dHraw,
    float* __restrict__ slab) {
  using C = AB3<U, NT>;
  constexpr int H2 = C::H2, NKS = C::NKS, MT = C::MT, NKS2 = C::NKS2, ROWS = C::ROWS, TOK = C::TOK;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, n = lane & 15;
  const int gw = blockIdx.x * AB3_WAVES + wave, nw = gridDim.x * AB3_WAVES;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u16x8_t* lA = reinterpret_cast<u16x8_t*>(smem);
  u16x8_t* lAT = lA + C::NA;
  float* lbw = reinterpret_cast<float*>(lAT + C::NA2);           // [b1 | w2] padded to ROWS each
  unsigned char* wbase = smem + C::HEAD + (size_t)wave * C::WAVE;
  unsigned short* dpi = reinterpret_cast<unsigned short*>(wbase + 2 * C::BUF);   // dP image [16][ROWS]
  for (int i = threadIdx.x; i < C::NA; i += 256) lA[i] = w1pack[i];
  for (int i = threadIdx.x; i < C::NA2; i += 256) lAT[i] = w1tpack[i];
  for (int i = threadIdx.x; i < ROWS; i += 256) {
    lbw[i] = i < H2 ? b1[i] : 0.f;
    lbw[ROWS + i] = i < H2 ? w2[i] : 0.f;
  }
  // zero the wave's buffers once: image rows >= L, alphas >= L and de >= H2 are never written by
  // the DMA and must read as 0 (padding tokens / features)
  for (int i = lane; i < C::WAVE / 16; i += 64) reinterpret_cast<uint4*>(wbase)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();

  // one sentence's rows -> buffer bf (wave-uniform); lanes past the data stay inactive
  const int hbytes = L * H2 * 2;
  auto prefetch = [&](int s, int bf) {
    unsigned char* bb = wbase + bf * C::BUF;
    const unsigned char* hs = reinterpret_cast<const unsigned char*>(hraw) + (size_t)s * hbytes;
    for (int k = 0; k * 1024 < hbytes; ++k)
      if (k * 1024 + lane * 16 < hbytes) lds_dma16(hs + k * 1024 + lane * 16, bb + k * 1024);
    if (lane < L) lds_dma4(alphas + (size_t)s * L + lane, bb + C::HIMG);
    if (lane < H2) lds_dma4(de + (size_t)s * H2 + lane, bb + C::HIMG + TOK * 4);
  };

  f32x4_t accW[MT][MT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < MT; ++b) accW[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dw2a[MT][4], db1a[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) dw2a[m][r] = db1a[m][r] = 0.f;
  // transposed-read lane roles: lane 4 q' + p of its 16-lane group g reads row (token) 4 g + q',
  // columns 4 p .. 4 p + 3 of a 4 x 16 block
  const int trow = 4 * q + ((lane & 15) >> 2), tcol = 4 * (lane & 3);

  int bf = 0;
  if (gw < S) prefetch(gw, 0);
  for (int s = gw; s < S; s += nw, bf ^= 1) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // this buffer landed; old reads done
    if (s + nw < S) prefetch(s + nw, bf ^ 1);
    const unsigned char* bb = wbase + bf * C::BUF;
    const unsigned short* img = reinterpret_cast<const unsigned short*>(bb);
    const float* alv_l = reinterpret_cast<const float*>(bb + C::HIMG);
    const float* de_l = reinterpret_cast<const float*>(bb + C::HIMG + TOK * 4);
    // ---- the sentence's operands from LDS (H tiles are re-read per pass: fewer live registers)
    auto ld_h = [&](int nt, u16x8_t* ht) __attribute__((always_inline)) {
      const int tok = 16 * nt + n;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int k0 = 32 * ks + 8 * q;
        const u16x8_t v = *reinterpret_cast<const u16x8_t*>(img + tok * H2 + (k0 < H2 ? k0 : 0));
        ht[ks] = k0 < H2 ? v : u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
    };
    float al[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) al[nt] = ldsf(alv_l + 16 * nt + n);   // 0 for tok >= L
    // ---- pass A: d(alpha)_t = de . H_t, sd = sum_t alpha_t d(alpha)_t
    float da[NT];
    float sd = 0.f;
    {
      float dev[NKS][8];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        ldsf4(de_l + 32 * ks + 8 * q, &dev[ks][0]);
        ldsf4(de_l + 32 * ks + 8 * q + 4, &dev[ks][4]);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        u16x8_t ht[NKS];
        ld_h(nt, ht);
        float d = 0.f;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) d += dev[ks][j] * bf2f(ht[ks][j]);
        da[nt] = cross_group_sum(d);
        sd += al[nt] * da[nt];
      }
    }
    sd = group16_sum(sd);
    // ---- pass B per 16-token tile (not unrolled; the tile's scalars picked with compile-time selects)
#pragma unroll 1
    for (int nt = 0; nt < NT; ++nt) {
      asm volatile("" ::: "memory");   // re-read the LDS operands per tile (no hoisting)
      u16x8_t ht[NKS];
      ld_h(nt, ht);
      float alv = al[0], dav = da[0];
#pragma unroll
      for (int j = 1; j < NT; ++j)
        if (j == nt) {
          alv = al[j];
          dav = da[j];
        }
      const int tok = 16 * nt + n;
      const float ds = alv * (dav - sd);   // 0 for padding tokens (alpha 0)
      float dp[MT][4];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float bj[4], wv[4];
        ldsf4(&lbw[16 * m + 4 * q], bj);
        ldsf4(&lbw[ROWS + 16 * m + 4 * q], wv);
        f32x4_t acc = {bj[0], bj[1], bj[2], bj[3]};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) acc = mfma_bf16(lA[(m * NKS + ks) * 64 + lane], ht[ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pr = tanhf_(acc[r]);
          dp[m][r] = ds * wv[r] * (1.f - pr * pr);
          dw2a[m][r] += ds * pr;
          db1a[m][r] += dp[m][r];
        }
      }
      u16x8_t B2[NKS2];
#pragma unroll
      for (int ks = 0; ks < NKS2; ++ks) {
        B2[ks] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int idx = ks * 8 + j;
          if (idx < 4 * MT) B2[ks][j] = f2bf(dp[idx >> 2][idx & 3]);
        }
      }
      unsigned short* dst = dHraw + ((size_t)s * L + (tok < L ? tok : 0)) * H2;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS2; ++ks) acc = mfma_bf16(lAT[(m * NKS2 + ks) * 64 + lane], B2[ks], acc);
        if (tok < L && 16 * m + 4 * q < H2) {
          uint2 pk;
          float dei[4];
          ldsf4(de_l + 16 * m + 4 * q, dei);
          pk.x = (uint32_t)f2bf(acc[0] + alv * dei[0]) | ((uint32_t)f2bf(acc[1] + alv * dei[1]) << 16);
          pk.y = (uint32_t)f2bf(acc[2] + alv * dei[2]) | ((uint32_t)f2bf(acc[3] + alv * dei[3]) << 16);
          *reinterpret_cast<uint2*>(dst + 16 * m + 4 * q) = pk;
        }
      }
      // dP tile -> [token n][j] image (8-B stores), then dW1 += H_tile^T dP_tile, K = the 16 tokens
#pragma unroll
      for (int m = 0; m < MT; ++m)
        *reinterpret_cast<u16x4_t*>(dpi + n * ROWS + 16 * m + 4 * q) =
            u16x4_t{f2bf(dp[m][0]), f2bf(dp[m][1]), f2bf(dp[m][2]), f2bf(dp[m][3])};
      lds_order();
      s16x4_t fb[MT];
#pragma unroll
      for (int b = 0; b < MT; ++b) fb[b] = tr_read(dpi + trow * ROWS + 16 * b + tcol);
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        // features 16 a + tcol .. + 3 of token 16 nt + trow (columns >= H2 read the next row: they only
        // feed dW1 rows >= H2, which are dropped)
        const s16x4_t fa = tr_read(img + (16 * nt + trow) * H2 + 16 * a + tcol);
#pragma unroll
        for (int b = 0; b < MT; ++b) accW[a][b] = mfma16_bf16(fa, fb[b], accW[a][b]);
      }
      lds_order();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA in flight into the reused LDS
  // ---- workgroup reduction into the slab (reuse the LDS as fp32 after a barrier)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  const int NS = H2 * H2 + 2 * H2;
  for (int i = threadIdx.x; i < NS; i += 256) red[i] = 0.f;
  __syncthreads();
  float d1s[MT][4], d2s[MT][4];   // cross-lane sums first (every lane takes part in the shuffles)
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d1s[m][r] = group16_sum(db1a[m][r]);
      d2s[m][r] = group16_sum(dw2a[m][r]);
    }
  ordered_wave_accumulate(threadIdx.x >> 6, 4, [&] {   // 256-thread workgroups; deterministic order
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < MT; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 16 * a + 4 * q + r, j = 16 * b + n;
          if (i < H2 && j < H2) red[i * H2 + j] += accW[a][b][r];
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
  for (int i = threadIdx.x; i < NS; i += 256) slab[(size_t)blockIdx.x * NS + i] = red[i];
}

// ------------------------------------------------------------------------------------------
namespace ina {



size_t attn_bwd_lds_bytes(int U, int NT, bool bf16) {
  const int H2 = 2 * U, MT = (H2 + 15) / 16;
  const int TOKP = ((NT * 16 + 31) / 32) * 32, RS = TOKP + (bf16 ? 8 : 4);
  size_t a = (size_t)4 * 2 * MT * 16 * RS * (bf16 ? 2 : 4);
  size_t r = (size_t)(H2 * H2 + 2 * H2) * 4;
  return a > r ? a : r;
}

template <int U, int NT, bool BF16>
static int attn_fwd_t(const AttnArgs& a, hipStream_t st) {
  using F = FT<BF16>;
  hipLaunchKernelGGL((attn_fwd_kernel<U, NT, BF16>), dim3(a.blocks), dim3(256), 0, st,
                     (const typename F::elem*)a.hraw, a.inst, a.mask, a.S, a.L, (const typename F::frag*)a.w1pack,
                     a.b1, a.w2, a.e, a.alphas);
  INA_CHECK_LAUNCH();
  return 0;
}
template <int U, int NT>
static size_t attn_bwd3_lds_bytes() {
  using C = AB3<U, NT>;
  const size_t b = (size_t)C::HEAD + (size_t)AB3_WAVES * C::WAVE;
  const size_t r = (size_t)(C::H2 * C::H2 + 2 * C::H2) * 4;
  return b > r ? b : r;
}

template <int U, int NT, bool BF16>
static int attn_bwd_t(const AttnArgs& a, hipStream_t st) {
  using F = FT<BF16>;
  if constexpr (BF16) {
    const size_t lds3 = attn_bwd3_lds_bytes<U, NT>();
    if (lds3 > 160 * 1024) return -1;
    if (lds3 > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<U, NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
    hipLaunchKernelGGL((attn_bwd3_kernel<U, NT>), dim3(a.blocks), dim3(256), lds3, st,
                       (const unsigned short*)a.hraw, a.S, a.L, (const u16x8_t*)a.w1pack,
                       (const u16x8_t*)a.w1tpack, a.b1, a.w2, a.de, a.alphas, (unsigned short*)a.dHraw, a.slab);
    INA_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = attn_bwd_lds_bytes(U, NT, BF16);
  hipLaunchKernelGGL((attn_bwd_kernel<U, NT, BF16>), dim3(a.blocks), dim3(256), lds, st,
                     (const typename F::elem*)a.hraw, a.inst, a.S, a.L, (const typename F::frag*)a.w1pack,
                     (const typename F::frag*)a.w1tpack, a.b1, a.w2, a.de, a.alphas, (typename F::elem*)a.dHraw, a.slab);
  INA_CHECK_LAUNCH();
  return 0;
}

#define INA_ATTN_CASE(FN, UU)                               \
  if (U == UU) {                                            \
    if (NT == 1) return FN<UU, 1, B>(a, st);                \
    if (NT == 2) return FN<UU, 2, B>(a, st);                \
    if (NT == 3) return FN<UU, 3, B>(a, st);                \
    if (NT == 4) return FN<UU, 4, B>(a, st);                \
  }
#define INA_ATTN_DISPATCH(FN)                 \
  if (bf16) {                                 \
    constexpr bool B = true;                  \
    INA_ATTN_CASE(FN, 8) INA_ATTN_CASE(FN, 20) INA_ATTN_CASE(FN, 32) \
  } else {                                    \
    constexpr bool B = false;                 \
    INA_ATTN_CASE(FN, 8) INA_ATTN_CASE(FN, 20) INA_ATTN_CASE(FN, 32) \
  }                                           \
  return -1;

// Workgroups of the persistent bf16 backward that are resident at once (occupancy x CUs): the grid
// is sized to exactly that, so every wave runs the same number of sentences in one round (a grid of
// 1024 at 3 workgroups per CU ran 1.33 rounds).  0 = unknown (fp32 kernel / query failed).
template <int U, int NT>
static int attn_bwd3_resident() {
  static int cached = -1;
  if (cached >= 0) return cached;
  const size_t lds3 = attn_bwd3_lds_bytes<U, NT>();
  if (lds3 > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<U, NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, attn_bwd3_kernel<U, NT>, 256, lds3) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    per_cu = cus = 0;
  cached = per_cu * cus;
  return cached;
}
int attn_bwd_resident_blocks(int U, int NT, bool bf16) {
  if (!bf16) return 0;
#define INA_AB3R(UV)                                 \
  if (U == UV) {                                     \
    if (NT == 1) return attn_bwd3_resident<UV, 1>(); \
    if (NT == 2) return attn_bwd3_resident<UV, 2>(); \
    if (NT == 3) return attn_bwd3_resident<UV, 3>(); \
    if (NT == 4) return attn_bwd3_resident<UV, 4>(); \
  }
  INA_AB3R(8) INA_AB3R(20) INA_AB3R(32)
#undef INA_AB3R
  return 0;
}

int attn_fwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st) { INA_ATTN_DISPATCH(attn_fwd_t) }
int attn_bwd(const AttnArgs& a, int U, int NT, bool bf16, hipStream_t st) { INA_ATTN_DISPATCH(attn_bwd_t) }

}  // namespace ina
