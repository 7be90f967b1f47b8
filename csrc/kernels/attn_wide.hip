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
// Both kernels are persistent (grid = resident workgroups, a loop over blocks): the W1 fragments are
// loaded once per workgroup instead of once per block (they were 2-4 GB of L2 traffic per step at the
// paper configuration), and every block's inputs (H rows, mask flags / alphas, de) are prefetched into
// registers while the previous block computes, so HBM latency is off the critical path.
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
  static constexpr int HS = HP + 16;   // LDS row stride (elements): rows 2 bank slots apart, so the MFMA
                                       // B-operand reads are conflict-free (lstm_wide.hip WideCfg)
  static constexpr int NTH = NW * 64;  // = 2 HP
  static constexpr int CP = HP / 8;    // 16-byte chunks per padded row
  static constexpr int PFH = 6;        // prefetched H chunks per thread: blocks of <= 96 tokens
  static constexpr int PFD = 2;        // prefetched de values per thread: SB <= 4
  static_assert(96 * CP == PFH * NTH, "prefetch slots cover a 96-token block");
};
constexpr int ATTN_PF_TOKENS = 96;

struct Blk {
  int s0, nseq, Tv, R, ntile;
};

INA_DEVICE Blk block_geom(int blk, int S, int L, int SB) {
  Blk b;
  b.s0 = blk * SB;
  b.nseq = min(SB, S - b.s0);
  b.Tv = b.nseq * L;
  b.ntile = (SB * L + 15) / 16;
  b.R = b.ntile * 16;
  return b;
}

// One block's inputs in registers (the next block's, loaded while the current one computes):
// H rows as 16-byte chunks (zero past the valid tokens / features), a per-token value (forward:
// the mask flag, backward: alpha) and the backward's de rows.
template <int HP, bool BWD>
struct Prefetch {
  using C = AttnCfg<HP>;
  u16x8_t h[C::PFH];
  float tv;
  float de[C::PFD];

  INA_DEVICE void load(const WideAttnArgs& a, const Blk& b) {
    const unsigned short* hin = reinterpret_cast<const unsigned short*>(a.hin);
    const int L = a.L, H = a.H, CH = H / 8;
    const size_t g0 = (size_t)b.s0 * L;
#pragma unroll
    for (int k = 0; k < C::PFH; ++k) {
      const int i = threadIdx.x + k * C::NTH, r = i / C::CP, ch = i - r * C::CP;
      h[k] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      if (r < b.Tv && ch < CH) h[k] = *reinterpret_cast<const u16x8_t*>(hin + (g0 + r) * H + 8 * ch);
    }
    const int tok = threadIdx.x;
    tv = 0.f;
    if (tok < b.Tv) {
      if (BWD) {
        tv = a.alpha[g0 + tok];
      } else {
        const int sl = tok / L, t = tok - sl * L;
        tv = a.mask[(size_t)a.inst[b.s0 + sl] * L + t] > 0 ? 1.f : 0.f;
      }
    }
    if (BWD) {
#pragma unroll
      for (int k = 0; k < C::PFD; ++k) {
        const int i = threadIdx.x + k * C::NTH, sl = i / HP, f = i - sl * HP;
        de[k] = sl < b.nseq && f < H ? a.de[(size_t)(b.s0 + sl) * H + f] : 0.f;
      }
    }
  }
  INA_DEVICE void store(const Blk& b, int SB, unsigned short* hb, float* tvs, float* deL) const {
#pragma unroll
    for (int k = 0; k < C::PFH; ++k) {
      const int i = threadIdx.x + k * C::NTH, r = i / C::CP, ch = i - r * C::CP;
      if (r < b.R) *reinterpret_cast<u16x8_t*>(hb + r * C::HS + 8 * ch) = h[k];
    }
    if ((int)threadIdx.x < b.R) tvs[threadIdx.x] = tv;
    if (BWD) {
#pragma unroll
      for (int k = 0; k < C::PFD; ++k) {
        const int i = threadIdx.x + k * C::NTH;
        if (i < SB * HP) deL[i] = de[k];
      }
    }
  }
};

// Blocks longer than the prefetch capacity (L > 96): stage straight from global memory.
template <int HP, bool BWD>
INA_DEVICE void stage_direct(const WideAttnArgs& a, const Blk& b, unsigned short* hb, float* tvs, float* deL) {
  using C = AttnCfg<HP>;
  const unsigned short* hin = reinterpret_cast<const unsigned short*>(a.hin);
  const int L = a.L, H = a.H, CH = H / 8;
  const size_t g0 = (size_t)b.s0 * L;
  for (int i = threadIdx.x; i < b.R * C::CP; i += C::NTH) {
    const int r = i / C::CP, ch = i - r * C::CP;
    u16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < b.Tv && ch < CH) v = *reinterpret_cast<const u16x8_t*>(hin + (g0 + r) * H + 8 * ch);
    *reinterpret_cast<u16x8_t*>(hb + r * C::HS + 8 * ch) = v;
  }
  for (int tok = threadIdx.x; tok < b.R; tok += C::NTH) {
    float v = 0.f;
    if (tok < b.Tv) {
      if (BWD) {
        v = a.alpha[g0 + tok];
      } else {
        const int sl = tok / L, t = tok - sl * L;
        v = a.mask[(size_t)a.inst[b.s0 + sl] * L + t] > 0 ? 1.f : 0.f;
      }
    }
    tvs[tok] = v;
  }
  if (BWD) {
    for (int i = threadIdx.x; i < a.SB * HP; i += C::NTH) {
      const int sl = i / HP, f = i - sl * HP;
      deL[i] = sl < b.nseq && f < H ? a.de[(size_t)(b.s0 + sl) * H + f] : 0.f;
    }
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

INA_DEVICE uint2 pack4_bf16(float a, float b, float c, float d) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t lo = {(__bf16)a, (__bf16)b}, hi = {(__bf16)c, (__bf16)d};
  return uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}

}  // namespace

template <int HP>
__global__ __launch_bounds__(AttnCfg<HP>::NTH) void wide_attn_fwd_kernel(WideAttnArgs a) {
  using C = AttnCfg<HP>;
  constexpr int NW = C::NW, HS = C::HS, NTH = C::NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S, L = a.L, H = a.H, SB = a.SB;
  const int nblk = (S + SB - 1) / SB;
  const int R = (SB * L + 15) / 16 * 16;
  const bool pf = R <= ATTN_PF_TOKENS;
  unsigned short* hb = reinterpret_cast<unsigned short*>(smem);        // [R][HS] bf16
  float* spart = reinterpret_cast<float*>(smem + (size_t)R * HS * 2);  // [NW][R] score partials
  float* alp = spart + NW * R;                                         // [R] mask flag -> score -> alpha
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, n = lane & 15;
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
  Prefetch<HP, false> nx;
  if (pf && (int)blockIdx.x < nblk) nx.load(a, block_geom(blockIdx.x, S, L, SB));
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const Blk b = block_geom(blk, S, L, SB);
    __syncthreads();   // the previous block is done with the LDS images
    if (pf) {
      nx.store(b, SB, hb, alp, nullptr);
      if (blk + (int)gridDim.x < nblk) nx.load(a, block_geom(blk + gridDim.x, S, L, SB));
    } else {
      stage_direct<HP, false>(a, b, hb, alp, nullptr);
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
      if (q == 0) spart[w * R + tile * 16 + n] = v;
    }
    __syncthreads();
    // masked softmax over each sequence's L positions (one wave per sequence)
    for (int sl = w; sl < b.nseq; sl += NW) {
      const int s = b.s0 + sl;
      float mx = -INFINITY;
      for (int t = lane; t < L; t += 64) {
        const int tok = sl * L + t;
        float sc = 0.f;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) sc += spart[ww * R + tok];
        sc = alp[tok] > 0.f ? sc : -INFINITY;
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
    // e = sum_t alpha_t H_t (fp32): one feature per thread (every wave busy: SB H = 512 at the paper
    // configuration), the token loop unrolled by 4 into independent partial sums so 4 tokens' LDS reads are
    // in flight (the two-features-per-thread serial loop left half the waves idle on a 37-step LDS-latency
    // chain per block)
    for (int i = threadIdx.x; i < b.nseq * H; i += NTH) {
      const int sl = i / H, f = i - sl * H;
      const unsigned short* hp = hb + (sl * L) * HS + f;
      const float* ap = alp + sl * L;
      float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
      int t = 0;
      for (; t + 4 <= L; t += 4) {
        e0 += ap[t] * bf2f(hp[t * HS]);
        e1 += ap[t + 1] * bf2f(hp[(t + 1) * HS]);
        e2 += ap[t + 2] * bf2f(hp[(t + 2) * HS]);
        e3 += ap[t + 3] * bf2f(hp[(t + 3) * HS]);
      }
      for (; t < L; ++t) e0 += ap[t] * bf2f(hp[t * HS]);
      a.e[(size_t)(b.s0 + sl) * H + f] = (e0 + e1) + (e2 + e3);
    }
  }
}

template <int HP>
__global__ __launch_bounds__(AttnCfg<HP>::NTH) void wide_attn_bwd_kernel(WideAttnArgs a) {
  // Register budget: W1^T and W1 fragments take 128 VGPRs, so the next block is streamed into a
  // second LDS image 32 rows per tile (2 chunks per thread, loaded before the tile's MFMAs and stored
  // after them) instead of being held in registers whole.
  using C = AttnCfg<HP>;
  constexpr int NW = C::NW, KS = C::KS, HS = C::HS, NTH = C::NTH, CP = C::CP;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int S = a.S, L = a.L, H = a.H, SB = a.SB, CH = H / 8;
  const int nblk = (S + SB - 1) / SB;
  const int R = (SB * L + 15) / 16 * 16;
  unsigned short* hbuf = reinterpret_cast<unsigned short*>(smem);               // [2][R][HS] bf16
  unsigned short* dzt = hbuf + 2 * (size_t)R * HS;                              // [2][16][HS] bf16
  float* debuf = reinterpret_cast<float*>(dzt + 2 * 16 * HS);                   // [2][SB][HP]
  float* abuf = debuf + 2 * SB * HP;                                            // [2][R] alphas
  float* dsv = abuf + 2 * R;                                                    // [R]
  float* bwj = dsv + R;                                                         // [2][HP]: b1 (pre-scaled), w2
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, n = lane & 15;
  u16x8_t A1[2][KS], A2[2][KS];
  load_frags<HP>(reinterpret_cast<const u16x8_t*>(a.w1t), w, lane, A1);
  load_frags<HP>(reinterpret_cast<const u16x8_t*>(a.w1), w, lane, A2);
  float gw2[2][4], gb1[2][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gw2[mt][r] = 0.f;
      gb1[mt][r] = 0.f;
    }
  for (int j = threadIdx.x; j < HP; j += NTH) {
    bwj[j] = a.b1[j] * (2.f * LOG2E_F);
    bwj[HP + j] = a.w2[j];
  }
  const unsigned short* hin = reinterpret_cast<const unsigned short*>(a.hin);
  unsigned short* dZg = reinterpret_cast<unsigned short*>(a.dZ);
  unsigned short* dHg = reinterpret_cast<unsigned short*>(a.dH);
  int cur = 0;
  if ((int)blockIdx.x < nblk) stage_direct<HP, true>(a, block_geom(blockIdx.x, S, L, SB), hbuf, abuf, debuf);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const Blk b = block_geom(blk, S, L, SB);
    const bool more = blk + (int)gridDim.x < nblk;
    const Blk nb = block_geom(more ? blk + gridDim.x : blk, S, L, SB);
    unsigned short* hb = hbuf + (size_t)cur * R * HS;
    unsigned short* hn = hbuf + (size_t)(cur ^ 1) * R * HS;
    float* deL = debuf + cur * SB * HP;
    float* alp = abuf + cur * R;
    // the next block's alphas / de rows: registers now, LDS after the last tile
    float tvn = 0.f, den[C::PFD];
    if (more) {
      if ((int)threadIdx.x < nb.Tv) tvn = a.alpha[(size_t)nb.s0 * L + threadIdx.x];
#pragma unroll
      for (int k = 0; k < C::PFD; ++k) {
        const int i = threadIdx.x + k * NTH, sl = i / HP, f = i - sl * HP;
        den[k] = sl < nb.nseq && f < H ? a.de[(size_t)(nb.s0 + sl) * H + f] : 0.f;
      }
    }
    __syncthreads();   // this block's images are complete; the previous block is done with the others
    // softmax backward, ds_t = alpha_t (de . H_t - sum_t' alpha_t' de . H_t'):
    // (1) da_t = de . H_t by all threads, 8 lanes per token (16-byte feature chunks c, c + 8, ..),
    //     combined with three xor-shuffles; padded tokens get 0
    for (int i = threadIdx.x; i < R * 8; i += NTH) {   // R * 8 is a multiple of 64: whole waves
      const int tok = i >> 3, c0 = i & 7, sl = min(tok / L, SB - 1);
      float d = 0.f;
      for (int c = c0; c < CP; c += 8) {
        const u16x8_t hv = *reinterpret_cast<const u16x8_t*>(hb + tok * HS + 8 * c);
        const float4 d0 = *reinterpret_cast<const float4*>(deL + sl * HP + 8 * c);
        const float4 d1 = *reinterpret_cast<const float4*>(deL + sl * HP + 8 * c + 4);
        d += d0.x * bf2f(hv[0]) + d0.y * bf2f(hv[1]) + d0.z * bf2f(hv[2]) + d0.w * bf2f(hv[3]) +
             d1.x * bf2f(hv[4]) + d1.y * bf2f(hv[5]) + d1.z * bf2f(hv[6]) + d1.w * bf2f(hv[7]);
      }
      d += __shfl_xor(d, 1);
      d += __shfl_xor(d, 2);
      d += __shfl_xor(d, 4);
      if (c0 == 0) dsv[tok] = tok < b.Tv ? d : 0.f;
    }
    __syncthreads();
    // (2) one wave per sequence: the alpha-weighted sum, then ds in place
    for (int sl = w; sl < b.nseq; sl += NW) {
      float acc = 0.f;
      for (int t = lane; t < L; t += 64) acc += alp[sl * L + t] * dsv[sl * L + t];
      const float tot = wave_sum(acc);
      for (int t = lane; t < L; t += 64) dsv[sl * L + t] = alp[sl * L + t] * (dsv[sl * L + t] - tot);
    }
    __syncthreads();
    const size_t g0 = (size_t)b.s0 * L, gn = (size_t)nb.s0 * L;
    for (int tile = 0; tile < b.ntile; ++tile) {
      // stream rows 32 tile .. 32 tile + 31 of the next block (2 chunks per thread)
      u16x8_t pf[2];
      bool pfv[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + k * NTH, r = 32 * tile + i / CP, ch = i % CP;
        pfv[k] = more && r < R;
        pf[k] = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        if (pfv[k] && r < nb.Tv && ch < CH) pf[k] = *reinterpret_cast<const u16x8_t*>(hin + (gn + r) * H + 8 * ch);
      }
      unsigned short* dz = dzt + (tile & 1) * 16 * HS;
      const int tok = tile * 16 + n;
      {
        f32x4_t acc[2];
        z_tile<HP>(hb, tile, n, q, A1, acc);
        const float ds = dsv[tok];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int j0 = 32 * w + 16 * mt + 4 * q;
          const float4 bv = *reinterpret_cast<const float4*>(bwj + j0), wv = *reinterpret_cast<const float4*>(bwj + HP + j0);
          const float bj[4] = {bv.x, bv.y, bv.z, bv.w}, wj[4] = {wv.x, wv.y, wv.z, wv.w};
          float g[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = tanh_l2(acc[mt][r] * (2.f * LOG2E_F) + bj[r]);
            g[r] = ds * wj[r] * (1.f - p * p);
            gw2[mt][r] += ds * p;
            gb1[mt][r] += g[r];
          }
          *reinterpret_cast<uint2*>(dz + n * HS + j0) = pack4_bf16(g[0], g[1], g[2], g[3]);
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
      {   // dH rows widened (ina_common.h widen: lane group q ends up with features 32w + 8q .. + 7 of its
          // token): one 16-byte store per lane, 16 tokens x 64 B per instruction instead of two 8-byte stores
          // per lane; all lanes take part in the swaps, padded tokens are not stored
        const int sl = min(tok / L, SB - 1);
        const float al = alp[tok];
        const int k0 = 32 * w + 4 * q;
        const float4 d0 = *reinterpret_cast<const float4*>(deL + sl * HP + k0);
        const float4 d1 = *reinterpret_cast<const float4*>(deL + sl * HP + k0 + 16);
        uint2 X = pack4_bf16(acc[0][0] + al * d0.x, acc[0][1] + al * d0.y, acc[0][2] + al * d0.z, acc[0][3] + al * d0.w);
        uint2 Y = pack4_bf16(acc[1][0] + al * d1.x, acc[1][1] + al * d1.y, acc[1][2] + al * d1.z, acc[1][3] + al * d1.w);
        widen(X, Y);
        const int kw = 32 * w + 8 * q;
        if (tok < b.Tv && kw < H) *reinterpret_cast<uint4*>(dHg + (g0 + tok) * H + kw) = uint4{X.x, X.y, Y.x, Y.y};
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + k * NTH, r = 32 * tile + i / CP, ch = i % CP;
        if (pfv[k]) *reinterpret_cast<u16x8_t*>(hn + r * HS + 8 * ch) = pf[k];
      }
    }
    if (more) {
      float* aln = abuf + (cur ^ 1) * R;
      float* den_l = debuf + (cur ^ 1) * SB * HP;
      if ((int)threadIdx.x < R) aln[threadIdx.x] = tvn;
#pragma unroll
      for (int k = 0; k < C::PFD; ++k) {
        const int i = threadIdx.x + k * NTH;
        if (i < SB * HP) den_l[i] = den[k];
      }
    }
    cur ^= 1;
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

int wide_attn_sb(int L) { return L >= 80 ? 1 : min(4, 80 / L); }   // ~80 tokens, <= 4 sequences per block

size_t wide_attn_smem(int H, int L, bool bwd) {
  const int HP = wide_attn_hp(H), HS = HP + 16, SB = wide_attn_sb(L), R = (SB * L + 15) / 16 * 16;
  if (!bwd) return (size_t)R * HS * 2 + (size_t)(HP / 32) * R * 4 + (size_t)R * 4;
  return 2 * (size_t)R * HS * 2 + 2 * 16 * (size_t)HS * 2 + 2 * (size_t)SB * HP * 4 + 3 * (size_t)R * 4 +
         2 * (size_t)HP * 4;
}

template <int HP>
static const void* attn_fn(bool bwd) {
  return bwd ? reinterpret_cast<const void*>(&wide_attn_bwd_kernel<HP>)
             : reinterpret_cast<const void*>(&wide_attn_fwd_kernel<HP>);
}

static const void* attn_fn_of(int HP, bool bwd) {
  switch (HP) {
    case 128: return attn_fn<128>(bwd);
    case 224: return attn_fn<224>(bwd);
    case 256: return attn_fn<256>(bwd);
    default: return nullptr;
  }
}

// persistent grid: the resident workgroups of the whole device (never more than the blocks)
int wide_attn_grid(int H, int L, int S, bool bwd) {
  const int HP = wide_attn_hp(H);
  const void* fn = attn_fn_of(HP, bwd);
  if (!fn || S <= 0) return 0;
  const size_t sm = wide_attn_smem(H, L, bwd);
  if (sm > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm) != hipSuccess)
    return -1;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, 2 * HP, sm) != hipSuccess || per < 1) per = 1;
  const int SB = wide_attn_sb(L), nblk = (S + SB - 1) / SB;
  return min(nblk, per * cus);
}

template <int HP>
static int attn_launch(const WideAttnArgs& a, int grid, bool bwd, hipStream_t st) {
  const size_t sm = wide_attn_smem(a.H, a.L, bwd);
  if (bwd) {
    hipLaunchKernelGGL(wide_attn_bwd_kernel<HP>, dim3(grid), dim3(AttnCfg<HP>::NTH), sm, st, a);
  } else {
    hipLaunchKernelGGL(wide_attn_fwd_kernel<HP>, dim3(grid), dim3(AttnCfg<HP>::NTH), sm, st, a);
  }
  INA_CHECK_LAUNCH();
  return 0;
}

static int attn_dispatch(const WideAttnArgs& a, int grid, bool bwd, hipStream_t st) {
  if (a.S <= 0) return 0;
  if (a.L < 1 || a.L > 256 || a.SB != wide_attn_sb(a.L) || grid < 1 || wide_attn_smem(a.H, a.L, bwd) > 160 * 1024)
    return -1;
  switch (wide_attn_hp(a.H)) {
    case 128: return attn_launch<128>(a, grid, bwd, st);
    case 224: return attn_launch<224>(a, grid, bwd, st);
    case 256: return attn_launch<256>(a, grid, bwd, st);
    default: return -1;
  }
}

int wide_attn_fwd(const WideAttnArgs& a, int grid, hipStream_t st) { return attn_dispatch(a, grid, false, st); }
int wide_attn_bwd(const WideAttnArgs& a, int grid, hipStream_t st) { return attn_dispatch(a, grid, true, st); }

}  // namespace ina
