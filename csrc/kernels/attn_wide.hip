// Self-attention pooling of the wide BiLSTM outputs (hidden 2u = H in {128, 200, 256}), fused.
//
// Reference: model/layer_module.py:49-98 (self_attention):
//   Z = H W1 + b1,  P = tanh(Z),  score_t = P_t . w2,  alpha = softmax_t(score + mask_adder),
//   e = sum_t alpha_t H_t.
// The round-2 wide path ran this as a bf16 GEMM plus ~7 fp32 elementwise / reduction passes over the
// [S, L, H] activations forward and ~12 backward (7.8 ms per step at the paper configuration, 44 % of
// the step).  Here one workgroup owns SB whole sequences (SB L tokens, ~80):
//   * the block's H rows are staged once in LDS (row stride HP + 8: 16 lanes reading 16 rows hit
//     distinct banks);
//   * Z^T = W1^T H^T runs on MFMA with W1^T as A fragments in VGPRs: wave w owns the 32 output
//     features 32w .. 32w + 31 (two 16-row M-tiles), the B operand is 16 tokens read from LDS;
//     tanh, the w2 dot and the sum over the 4 lane groups happen on the accumulators; per-wave score
//     partials meet in LDS;
//   * softmax (one wave per sequence) and the alpha-weighted pooling read the same LDS image.
// Backward recomputes Z from the staged block instead of storing P (memory, not MFMA, is the bound):
//   ds_t = alpha_t (de . H_t - sum_t' alpha_t' de . H_t'),  dZ = ds w2 (1 - P^2),
//   dH = alpha de + dZ W1^T   (second MFMA pass, W1 as A fragments, dZ tile through LDS),
//   dw2 / db1: per-lane sums -> one partial row per workgroup; dZ (bf16) is written for the
//   dW1 = H^T dZ split-K GEMM (ops/wide.py).
// Operand layouts are built by ops/packing.py::pack_attn_wide and checked against the fp32 oracle
// by tests/test_wide_gpu.py.
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

template <int HP>
struct AttnCfg {
  static constexpr int NW = HP / 32;   // waves: two 16-feature M-tiles each
  static constexpr int KS = HP / 32;   // K-steps over the features
  static constexpr int HS = HP + 8;    // LDS row stride (elements)
  static constexpr int NTH = NW * 64;
};

struct Blk {
  int s0, nseq, Tv, R, ntile;
};

INA_DEVICE Blk block_geom(int S, int L, int SB) {
  Blk b;
  b.s0 = blockIdx.x * SB;
  b.nseq = min(SB, S - b.s0);
  b.Tv = b.nseq * L;
  b.ntile = (SB * L + 15) / 16;
  b.R = b.ntile * 16;
  return b;
}

// H rows of the block -> LDS [R][HS] (zero rows past the valid tokens, zero feature padding)
template <int HP>
INA_DEVICE void stage_block(const unsigned short* __restrict__ hin, int H, const Blk& b, int L,
                            unsigned short* hb) {
  using C = AttnCfg<HP>;
  constexpr int CP = HP / 8;
  const int CH = H / 8;
  const size_t g0 = (size_t)b.s0 * L;
  for (int i = threadIdx.x; i < b.R * CP; i += C::NTH) {
    const int r = i / CP, ch = i - r * CP;
    u16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < b.Tv && ch < CH) v = *reinterpret_cast<const u16x8_t*>(hin + (g0 + r) * H + 8 * ch);
    *reinterpret_cast<u16x8_t*>(hb + r * C::HS + 8 * ch) = v;
  }
}

template <int HP>
INA_DEVICE void load_frags(const u16x8_t* __restrict__ pk, int w, int lane, u16x8_t (&A)[2][AttnCfg<HP>::KS]) {
  constexpr int KS = AttnCfg<HP>::KS;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) A[mt][ks] = pk[((2 * w + mt) * KS + ks) * 64 + lane];
}

// Z^T for 16 tokens (rows tile*16 ..) and the wave's 32 features: acc[mt][r] = Z[token n][32w + 16mt + 4q + r]
template <int HP>
INA_DEVICE void z_tile(const unsigned short* hb, int tile, int n, int q, const u16x8_t (&A)[2][AttnCfg<HP>::KS],
                       f32x4_t (&acc)[2]) {
  using C = AttnCfg<HP>;
  acc[0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks) {
    const u16x8_t B = *reinterpret_cast<const u16x8_t*>(hb + (tile * 16 + n) * C::HS + 32 * ks + 8 * q);
    acc[0] = mfma_bf16(A[0][ks], B, acc[0]);
    acc[1] = mfma_bf16(A[1][ks], B, acc[1]);
  }
}

}  // namespace

template <int HP>
__global__ __launch_bounds__(AttnCfg<HP>::NTH) void wide_attn_fwd_kernel(WideAttnArgs a) {
  using C = AttnCfg<HP>;
  constexpr int NW = C::NW, HS = C::HS, NTH = C::NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int L = a.L, H = a.H;
  const Blk b = block_geom(a.S, L, a.SB);
  unsigned short* hb = reinterpret_cast<unsigned short*>(smem);          // [R][HS] bf16
  float* spart = reinterpret_cast<float*>(smem + (size_t)b.R * HS * 2);  // [NW][R] score partials
  float* alp = spart + NW * b.R;                                         // [R]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, n = lane & 15;
  stage_block<HP>(reinterpret_cast<const unsigned short*>(a.hin), H, b, L, hb);
  u16x8_t A[2][C::KS];
  load_frags<HP>(reinterpret_cast<const u16x8_t*>(a.w1t), w, lane, A);
  float bj[2][4], wj[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 32 * w + 16 * mt + 4 * q + r;
      bj[mt][r] = a.b1[j] * (2.f * LOG2E_F);
      wj[mt][r] = a.w2[j];
    }
  __syncthreads();
  for (int tile = 0; tile < b.ntile; ++tile) {
    f32x4_t acc[2];
    z_tile<HP>(hb, tile, n, q, A, acc);
    float v = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) v += wj[mt][r] * tanh_l2(acc[mt][r] * (2.f * LOG2E_F) + bj[mt][r]);
    v = cross_group_sum(v);
    if (q == 0) spart[w * b.R + tile * 16 + n] = v;
  }
  __syncthreads();
  // masked softmax over each sequence's L positions (one wave per sequence)
  for (int sl = w; sl < b.nseq; sl += NW) {
    const int s = b.s0 + sl;
    const int* mrow = a.mask + (size_t)a.inst[s] * L;
    float mx = -INFINITY;
    for (int t = lane; t < L; t += 64) {
      const int tok = sl * L + t;
      float sc = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sc += spart[ww * b.R + tok];
      sc = mrow[t] > 0 ? sc : -INFINITY;
      alp[tok] = sc;
      mx = fmaxf(mx, sc);
    }
    mx = wave_max(mx);
    float sum = 0.f;
    for (int t = lane; t < L; t += 64) {
      const int tok = sl * L + t;
      const float ex = alp[tok] == -INFINITY ? 0.f : __expf(alp[tok] - mx);
      alp[tok] = ex;
      sum += ex;
    }
    const float inv = 1.f / wave_sum(sum);
    for (int t = lane; t < L; t += 64) {
      const int tok = sl * L + t;
      const float al = alp[tok] * inv;
      alp[tok] = al;
      a.alpha[(size_t)s * L + t] = al;
    }
  }
  __syncthreads();
  // e = sum_t alpha_t H_t (fp32), two features per thread
  const int H2 = H / 2;
  for (int i = threadIdx.x; i < b.nseq * H2; i += NTH) {
    const int sl = i / H2, f = 2 * (i - sl * H2);
    float e0 = 0.f, e1 = 0.f;
    for (int t = 0; t < L; ++t) {
      const int tok = sl * L + t;
      const float al = alp[tok];
      const uint32_t hv = *reinterpret_cast<const uint32_t*>(hb + tok * HS + f);
      e0 += al * bf2f((unsigned short)hv);
      e1 += al * bf2f((unsigned short)(hv >> 16));
    }
    *reinterpret_cast<float2*>(a.e + (size_t)(b.s0 + sl) * H + f) = float2{e0, e1};
  }
}

template <int HP>
__global__ __launch_bounds__(AttnCfg<HP>::NTH) void wide_attn_bwd_kernel(WideAttnArgs a) {
  using C = AttnCfg<HP>;
  constexpr int NW = C::NW, KS = C::KS, HS = C::HS, NTH = C::NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int L = a.L, H = a.H, SB = a.SB;
  const Blk b = block_geom(a.S, L, SB);
  unsigned short* hb = reinterpret_cast<unsigned short*>(smem);                 // [R][HS] bf16
  unsigned short* dzt = hb + (size_t)b.R * HS;                                  // [2][16][HS] bf16
  float* deL = reinterpret_cast<float*>(dzt + 2 * 16 * HS);                     // [SB][HP]
  float* alp = deL + SB * HP;                                                   // [R]
  float* dsv = alp + b.R;                                                       // [R]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, n = lane & 15;
  stage_block<HP>(reinterpret_cast<const unsigned short*>(a.hin), H, b, L, hb);
  for (int i = threadIdx.x; i < b.R; i += NTH) alp[i] = i < b.Tv ? a.alpha[(size_t)b.s0 * L + i] : 0.f;
  for (int i = threadIdx.x; i < SB * HP; i += NTH) {
    const int sl = i / HP, f = i - sl * HP;
    deL[i] = sl < b.nseq && f < H ? a.de[(size_t)(b.s0 + sl) * H + f] : 0.f;
  }
  u16x8_t A1[2][KS], A2[2][KS];
  load_frags<HP>(reinterpret_cast<const u16x8_t*>(a.w1t), w, lane, A1);
  load_frags<HP>(reinterpret_cast<const u16x8_t*>(a.w1), w, lane, A2);
  float bj[2][4], wj[2][4], gw2[2][4], gb1[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 32 * w + 16 * mt + 4 * q + r;
      bj[mt][r] = a.b1[j] * (2.f * LOG2E_F);
      wj[mt][r] = a.w2[j];
      gw2[mt][r] = 0.f;
      gb1[mt][r] = 0.f;
    }
  __syncthreads();
  // softmax backward: ds_t = alpha_t (de . H_t - sum_t' alpha_t' de . H_t'), one wave per sequence
  for (int sl = w; sl < SB; sl += NW) {
    float da[4];   // L <= 256 (host check): up to 4 positions per lane
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = lane + 64 * k;
      da[k] = 0.f;
      if (t < L && sl < b.nseq) {
        const int tok = sl * L + t;
        float d = 0.f;
        for (int f = 0; f < H; f += 2) {
          const uint32_t hv = *reinterpret_cast<const uint32_t*>(hb + tok * HS + f);
          d += deL[sl * HP + f] * bf2f((unsigned short)hv) + deL[sl * HP + f + 1] * bf2f((unsigned short)(hv >> 16));
        }
        da[k] = d;
        acc += alp[tok] * d;
      }
    }
    const float tot = wave_sum(acc);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = lane + 64 * k;
      if (t < L) {
        const int tok = sl * L + t;
        dsv[tok] = alp[tok] * (da[k] - tot);   // zero for padded / absent sequences (alpha = 0)
      }
    }
  }
  for (int i = SB * L + threadIdx.x; i < b.R; i += NTH) dsv[i] = 0.f;
  __syncthreads();
  const size_t g0 = (size_t)b.s0 * L;
  unsigned short* dZg = reinterpret_cast<unsigned short*>(a.dZ);
  unsigned short* dHg = reinterpret_cast<unsigned short*>(a.dH);
  constexpr int CP = HP / 8;
  const int CH = H / 8;
  for (int tile = 0; tile < b.ntile; ++tile) {
    unsigned short* dz = dzt + (tile & 1) * 16 * HS;
    const int tok = tile * 16 + n;
    {
      f32x4_t acc[2];
      z_tile<HP>(hb, tile, n, q, A1, acc);
      const float ds = dsv[tok];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        float g[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = tanh_l2(acc[mt][r] * (2.f * LOG2E_F) + bj[mt][r]);
          g[r] = ds * wj[mt][r] * (1.f - p * p);
          gw2[mt][r] += ds * p;
          gb1[mt][r] += g[r];
        }
        typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
        const bf2_t lo = {(__bf16)g[0], (__bf16)g[1]}, hi = {(__bf16)g[2], (__bf16)g[3]};
        *reinterpret_cast<uint2*>(dz + n * HS + 32 * w + 16 * mt + 4 * q) =
            uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
      }
    }
    __syncthreads();   // the dZ tile is complete (double-buffered: one barrier per tile)
    // dZ rows -> global (the dW1 GEMM operand), coalesced 16-byte chunks
    for (int i = threadIdx.x; i < 16 * CP; i += NTH) {
      const int rr = i / CP, ch = i - rr * CP, t2 = tile * 16 + rr;
      if (t2 < b.Tv && ch < CH)
        *reinterpret_cast<u16x8_t*>(dZg + (g0 + t2) * H + 8 * ch) = *reinterpret_cast<const u16x8_t*>(dz + rr * HS + 8 * ch);
    }
    // dH^T[k][token] = sum_j W1[k][j] dZ[token][j] + alpha_token de[k]; the wave's k = 32w + 16mt + 4q + r
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8_t B = *reinterpret_cast<const u16x8_t*>(dz + n * HS + 32 * ks + 8 * q);
      acc[0] = mfma_bf16(A2[0][ks], B, acc[0]);
      acc[1] = mfma_bf16(A2[1][ks], B, acc[1]);
    }
    if (tok < b.Tv) {
      const int sl = tok / L;
      const float al = alp[tok];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int k0 = 32 * w + 16 * mt + 4 * q;
        if (k0 < H) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[mt][r] + al * deL[sl * HP + k0 + r];
          typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
          const bf2_t lo = {(__bf16)v[0], (__bf16)v[1]}, hi = {(__bf16)v[2], (__bf16)v[3]};
          *reinterpret_cast<uint2*>(dHg + (g0 + tok) * H + k0) =
              uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
        }
      }
    }
  }
  // dw2 / db1 partials of this workgroup: sum over the 16 token lanes, one row per workgroup
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s2 = group16_sum(gw2[mt][r]), s1 = group16_sum(gb1[mt][r]);
      if (n == 0) {
        const int j = 32 * w + 16 * mt + 4 * q + r;
        a.part[(size_t)blockIdx.x * 2 * HP + j] = s2;
        a.part[(size_t)blockIdx.x * 2 * HP + HP + j] = s1;
      }
    }
}

namespace ina {

int wide_attn_hp(int H) { return (H == 128 || H == 200 || H == 256) ? (H + 31) / 32 * 32 : 0; }

size_t wide_attn_smem(int H, int L, int SB, bool bwd) {
  const int HP = wide_attn_hp(H), HS = HP + 8, R = (SB * L + 15) / 16 * 16;
  if (!bwd) return (size_t)R * HS * 2 + (size_t)(HP / 32) * R * 4 + (size_t)R * 4;
  return (size_t)R * HS * 2 + 2 * 16 * (size_t)HS * 2 + (size_t)SB * HP * 4 + 2 * (size_t)R * 4;
}

template <int HP>
static int attn_launch(const WideAttnArgs& a, bool bwd, hipStream_t st) {
  const dim3 grid((a.S + a.SB - 1) / a.SB);
  const size_t sm = wide_attn_smem(a.H, a.L, a.SB, bwd);
  const void* fn = bwd ? reinterpret_cast<const void*>(&wide_attn_bwd_kernel<HP>)
                       : reinterpret_cast<const void*>(&wide_attn_fwd_kernel<HP>);
  if (sm > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess)
    return -1;
  if (bwd) {
    hipLaunchKernelGGL(wide_attn_bwd_kernel<HP>, grid, dim3(AttnCfg<HP>::NTH), sm, st, a);
  } else {
    hipLaunchKernelGGL(wide_attn_fwd_kernel<HP>, grid, dim3(AttnCfg<HP>::NTH), sm, st, a);
  }
  INA_CHECK_LAUNCH();
  return 0;
}

static int attn_dispatch(const WideAttnArgs& a, bool bwd, hipStream_t st) {
  if (a.S <= 0) return 0;
  if (a.L < 1 || a.L > 256 || a.SB < 1 || wide_attn_smem(a.H, a.L, a.SB, bwd) > 160 * 1024) return -1;
  switch (wide_attn_hp(a.H)) {
    case 128: return attn_launch<128>(a, bwd, st);
    case 224: return attn_launch<224>(a, bwd, st);
    case 256: return attn_launch<256>(a, bwd, st);
    default: return -1;
  }
}

int wide_attn_fwd(const WideAttnArgs& a, hipStream_t st) { return attn_dispatch(a, false, st); }
int wide_attn_bwd(const WideAttnArgs& a, hipStream_t st) { return attn_dispatch(a, true, st); }

}  // namespace ina
