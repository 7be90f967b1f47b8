// Fused neural-tensor-layer relation module (K7 + K8 of SURVEY 2.3), bf16 MFMA, fp32 accumulate.
//
// Reference (model/layer_module.py:8-47, model/graph.py:81-86):
//   for s in 0..h-1:  S_s = (C @ M[:,:,s]) @ Q^T          [N, NQ]
//   V = relu(concat_s(S_s)^T)  with column index s*N + c   [NQ, h*N]
//   probs = sigmoid(V @ w + b),  w [h*N, N], b [N]        ("reference" head)
// "paper" head (paper Eq.11): probs[q, c] = sigmoid(sum_s w_s relu(T[q, s, c]) + b).
//
// Tile formulation.  The h slices are cut into tiles of SG = 16 / N slices (<= 4) so that the rows
// (slice, class) of one tile fill a 16-row MFMA operand (N = 5: 3 slices, 15 rows); a wave owns G = 2
// episodes (<= 16 / N) whose class rows (g, c) are stacked the same way.  Per tile:
//   P^T_s[b, (g,c)] = M_s^T C^T                 stacked over the wave's episodes (the dense product: 2x fewer
//                                               MFMAs than one episode per wave), written to a per-episode
//                                               LDS image P_g[(s,c)][b]
//   T^T_g[(s,c), q] = P_g Q_g^T                 A = P image rows (ds_read_b128), B = Q rows (registers)
//   fwd: logits^T[c', q] += Wt[c', (s,c)] relu(T^T)        16x16x16: the T^T accumulator IS the B operand
//   bwd: dV^T = W[(s,c), c'] dz^T; dT^T = [T > 0] dV^T      16x16x16: dz^T is the B operand
//        dw[(s,c), c'] += V dz                 A = V through a wave-private LDS image + ds_read_b64_tr_b16
//        dQ^T_g[b, q] += P_g^T dT^T             A = the P image read transposed (tr_b16), B = dT^T accumulator
//        dP^T_g[b, (s,c)] = Q^T dT              B = dT through an LDS image (tr_b16); dP -> global (dM GEMM)
//                                               and -> the P image's rows (the P image is dead by then)
//        dC^T[a, (g,c)] += M_s D_s              stacked over the wave's episodes again, B = the dP images
// Compared with one wave per episode and the rows (c) of every product padded to 16 this is 11 MFMAs per
// (slice, episode) in the backward instead of 25 (4 instead of 11 in the forward).
//
// A workgroup is 8 waves = 16 episodes.  The tile pack (M images + FC fragments, ops/packing.py::
// pack_ntn_tiles) is staged once per workgroup with global_load_lds (double buffered, one barrier per tile).
// LDS images are XOR-swizzled in 8-byte chunks (M: chunk ^ ((a & 2) << 1 | (a & 8)); P: chunk ^ ((r & 6) << 1);
// V / dT: a row-slot rotation), which makes the fragment reads of every product conflict-free.
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

constexpr int NW = 8;                // waves (each G episodes) per workgroup
constexpr int NT_THREADS = NW * 64;
constexpr int IMG_ROW = 128;         // bytes per LDS image row: 64 bf16
constexpr int PIMG = 16 * IMG_ROW + 64;   // per-episode P image [16 rows (slice, class)][64 b], + 64 B: the
                                         // two episodes' images sit 16 banks apart (their rows meet in one
                                         // write / read instruction)
constexpr int ZERO_BYTES = 256;      // zero block: the fragment reads of rows outside an image
constexpr int DW_SLOT = 256;         // floats per wave of the dw tile exchange
constexpr f32x4_t Z4 = {0.f, 0.f, 0.f, 0.f};
constexpr s16x4_t Z4S = {0, 0, 0, 0};

// M image row a: 8-byte chunk XOR {0,0,4,4,8,8,12,12,10,10,14,14,2,2,6,6}[a & 15] -- linear in the row bits,
// found exhaustively with the bank model (tools/lds_probe/mimage_search.py): the transposed full-K reads, the
// transposed 16-deep tail reads and the dC row reads are all conflict-free
INA_DEVICE int mask_m(int a) { return (int)((0x6622EEAACC884400ull >> (4 * (a & 15))) & 15u); }
// P image row r: 8-byte chunk XOR {0,4,12,2,10,14,6,8}[r & 7] (searched with an LDS bank model -- reads 64 banks,
// writes 32 banks per 16-lane group: the row reads, the transposed reads and the per-row stores are
// conflict-free, the stacked-episode stores 2-way; the (r & 6) << 1 mask had 4-way stores)
INA_DEVICE int mask_p(int r) { return (int)((0x86EA2C40u >> (4 * (r & 7))) & 15u); }
INA_DEVICE int vslot(int r) { return (r & ~15) | (r & 8) | ((r + ((r & 8) >> 1)) & 7); }
// V / dT image: byte offset of 8-byte chunk c of row r (row slots rotated, chunks XOR-ed by slot >> 2)
INA_DEVICE int voff(int r, int c) {
  const int sl = vslot(r);
  return sl * 32 + ((c ^ ((sl >> 2) & 3)) << 3);
}

INA_DEVICE s16x4_t trr(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)p);
}
INA_DEVICE u16x8_t cat8(const s16x4_t& lo, const s16x4_t& hi) {
  return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                 (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
}
// A 16-deep K tail accumulated onto 16x16x32 results: v_mfma_f32_16x16x32_bf16 with the upper half of both
// operands zero (same k relabelling on A and B, so the sum is the 16x16x16 product).  A back-to-back
// v_mfma_f32_16x16x32_bf16 -> v_mfma_f32_16x16x16_bf16 accumulate chain gets no wait states from hipcc (ROCm
// 7.2) and reads a stale SrcC on gfx950 (tools/lds_probe/mfma_chain.hip); the 16x16x16 form is no faster here
// (tools/lds_probe/mfma_rate.hip), so every chain keeps one opcode.
INA_DEVICE f32x4_t mfma_tail(const s16x4_t& a, const s16x4_t& b, const f32x4_t& c) {
  return mfma_bf16(cat8(a, Z4S), cat8(b, Z4S), c);
}
INA_DEVICE s16x4_t bf4(const f32x4_t& x) {
  return s16x4_t{(short)f2bf(x[0]), (short)f2bf(x[1]), (short)f2bf(x[2]), (short)f2bf(x[3])};
}
// relu on the packed bf16 values: a negative bf16 is a negative int16, so one v_pk_max_i16 per pair (fmaxf on
// the fp32 values costs a canonicalizing v_max plus the v_max per element)
INA_DEVICE s16x4_t bf4relu(const f32x4_t& x) {
  return __builtin_elementwise_max(bf4(x), Z4S);
}
// Unconditional load from a clamped index, zero outside (a lane-dependent branch around each load made
// hipcc wait vmcnt(0) per element); multiply rather than select so LLVM cannot sink the load under a branch
INA_DEVICE float ldz(const float* __restrict__ p, bool ok, long idx) { return p[ok ? idx : 0] * (ok ? 1.f : 0.f); }
// 4 consecutive floats p[idx .. idx + 3] (idx % 4 == 0) -> bf16 elements j0 .. j0 + 3 of f (zeros if !ok)
INA_DEVICE void ld4bf(const float* __restrict__ p, bool ok, long idx, u16x8_t& f, int j0) {
  const float4 v = *reinterpret_cast<const float4*>(p + (ok ? idx : 0));
  const float z = ok ? 1.f : 0.f;
  f[j0] = f2bf(v.x * z);
  f[j0 + 1] = f2bf(v.y * z);
  f[j0 + 2] = f2bf(v.z * z);
  f[j0 + 3] = f2bf(v.w * z);
}

// tile pack -> LDS: 1-KiB fragments, wave w takes fragments w, w + NW, ...
INA_DEVICE void stage_tile(unsigned char* dst, const unsigned char* __restrict__ src, int nfrag) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(dst));
  for (int f = wave; f < nfrag; f += NW) glds16_asm(src + (long)f * 1024 + lane * 16, base + f * 1024);
}
INA_DEVICE void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Order point of a wave's own cross-lane LDS traffic (lanes read what other lanes wrote): the wave's image
// base offset goes through an empty asm, so the compiler can prove no access after it disjoint from one
// before it.  No "memory" clobber: with one (or a fence) hipcc waits for the in-flight tile DMA (vmcnt(0))
// before every later LDS read.  The hardware runs a wave's LDS instructions in order.
// The lane index through an empty asm at the top of each tile: the lane-dependent LDS / global addresses
// are recomputed per tile (a few VALU) instead of being hoisted out of both loops into ~100 live registers.
INA_DEVICE int opaque_lane() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
INA_DEVICE void wave_order(uint32_t& off) {
  asm volatile("" : "+v"(off));
  __builtin_amdgcn_wave_barrier();
}

struct Geo {   // per-launch geometry shared by both kernels
  int N, NQ, G, SG, H, lg, lc;
  bool lrow;   // this lane's stacked class row (g, c) = (lg, lc) exists
};
INA_DEVICE Geo geo(const NtnArgs& k, int n) {
  Geo g;
  g.N = k.N;
  g.NQ = k.N * k.Q;
  g.G = k.G;
  g.SG = k.SG;
  g.H = k.H;
  g.lg = n / k.N;
  g.lc = n - g.lg * k.N;
  g.lrow = n < k.G * k.N;
  return g;
}

// C^T as the B operand of P^T (col = the lane's stacked row (g, c)): KF = MTH / 2 32-deep K-steps over a
// (16x16x32) and, for odd MTH, a 16-deep tail a = 32 KF .. + 15 (16x16x16; same cycles, half the LDS reads,
// and no reads of image rows past 16 MTH)
template <int MTH>
struct CFrag {
  static constexpr int KF = MTH / 2, TAIL = MTH & 1;
  u16x8_t f[KF > 0 ? KF : 1];
  s16x4_t t;
};
template <int MTH>
INA_DEVICE void load_cf(const NtnArgs& k, const Geo& g, int epw, int q, CFrag<MTH>& C) {
  const int ep = epw + g.lg;
  const bool ok = g.lrow && ep < k.E;
  const long row = (long)(ok ? ep : 0) * g.N + g.lc;
#pragma unroll
  for (int ka = 0; ka < CFrag<MTH>::KF; ++ka)
#pragma unroll
    for (int h4 = 0; h4 < 2; ++h4) {
      const int a = 32 * ka + 8 * q + 4 * h4;
      ld4bf(k.cls, ok && a < g.H, row * g.H + a, C.f[ka], 4 * h4);
    }
  if (CFrag<MTH>::TAIL) {
    u16x8_t t8;
    const int a = 32 * CFrag<MTH>::KF + 4 * q;
    ld4bf(k.cls, ok && a < g.H, row * g.H + a, t8, 0);
    C.t = s16x4_t{(short)t8[0], (short)t8[1], (short)t8[2], (short)t8[3]};
  } else {
    C.t = Z4S;
  }
}
// Q^T as the B operand of T^T: B[k = b][col = query 16 qt + n]; K over b as in CFrag (full steps + 16-deep tail)
template <int MTH, int QT>
struct QFrag {
  static constexpr int KF = MTH / 2, TAIL = MTH & 1;
  u16x8_t f[QT][KF > 0 ? KF : 1];
  s16x4_t t[QT];
};
template <int MTH, int QT>
INA_DEVICE void load_qf(const NtnArgs& k, const Geo& g, int ep, bool oke, int q, int n, QFrag<MTH, QT>& Qf) {
  const long rq0 = (long)(oke ? ep : 0) * (g.N * k.K + g.NQ) + g.N * k.K;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int qi = 16 * qt + n;
#pragma unroll
    for (int kb = 0; kb < QFrag<MTH, QT>::KF; ++kb)
#pragma unroll
      for (int h4 = 0; h4 < 2; ++h4) {
        const int b = 32 * kb + 8 * q + 4 * h4;
        ld4bf(k.e, oke && qi < g.NQ && b < g.H, (rq0 + qi) * g.H + b, Qf.f[qt][kb], 4 * h4);
      }
    if (QFrag<MTH, QT>::TAIL) {
      u16x8_t t8;
      const int b = 32 * QFrag<MTH, QT>::KF + 4 * q;
      ld4bf(k.e, oke && qi < g.NQ && b < g.H, (rq0 + qi) * g.H + b, t8, 0);
      Qf.t[qt] = s16x4_t{(short)t8[0], (short)t8[1], (short)t8[2], (short)t8[3]};
    } else {
      Qf.t[qt] = Z4S;
    }
  }
}

// P^T_s for the SG slices of the staged tile (stacked over the wave's episodes) -> the P images
template <int MTH, int SG>
INA_DEVICE void p_images(const unsigned char* buf, unsigned char* pimg, const Geo& g, const CFrag<MTH>& C, int q,
                         int n) {
  constexpr int RA = 16 * MTH, KF = CFrag<MTH>::KF;
  // lane offsets: the full steps read rows 32 ka + 8 q + (n >> 2) (lo) and + 4 (hi), the tail rows
  // 32 KF + 4 q + (n >> 2).  mask_m depends on the row bits 1..3 only (same for every ka / sl); the chunk
  // (4 mb + (n & 3)) ^ m splits into the 32-byte block mb ^ (m >> 2) and the 8-byte chunk (n & 3) ^ (m & 3)
  const int af = 8 * q + (n >> 2), at = 32 * KF + 4 * q + (n >> 2);
  const int ml = mask_m(af), mh = mask_m(af + 4), mt = mask_m(at);
  const int bl = af * IMG_ROW + (((n & 3) ^ (ml & 3)) << 3), bh = (af + 4) * IMG_ROW + (((n & 3) ^ (mh & 3)) << 3);
  const int bt = at * IMG_ROW + (((n & 3) ^ (mt & 3)) << 3);
#pragma unroll
  for (int sl = 0; sl < SG; ++sl) {
    const unsigned char* mimg = buf + sl * (RA * IMG_ROW);
    f32x4_t PT[MTH];
#pragma unroll
    for (int mb = 0; mb < MTH; ++mb) PT[mb] = Z4;
#pragma unroll
    for (int mb = 0; mb < MTH; ++mb) {
      const unsigned char* pl = mimg + bl + 32 * (mb ^ (ml >> 2));
      const unsigned char* ph = mimg + bh + 32 * (mb ^ (mh >> 2));
#pragma unroll
      for (int ka = 0; ka < KF; ++ka)
        PT[mb] = mfma_bf16(cat8(trr(pl + ka * 32 * IMG_ROW), trr(ph + ka * 32 * IMG_ROW)), C.f[ka], PT[mb]);
      if (CFrag<MTH>::TAIL) PT[mb] = mfma_tail(trr(mimg + bt + 32 * (mb ^ (mt >> 2))), C.t, PT[mb]);
    }
    if (g.lrow) {
      const int row = sl * g.N + g.lc;
      unsigned char* dst = pimg + g.lg * PIMG + row * IMG_ROW;
#pragma unroll
      for (int mb = 0; mb < MTH; ++mb)
        *reinterpret_cast<s16x4_t*>(dst + (((4 * mb + q) ^ mask_p(row)) << 3)) = bf4(PT[mb]);
    }
  }
}

// A = P_g[i = (s,c) = n][k = b]: the full 32-deep K-steps (ds_read_b128) and the 16-deep tail (ds_read_b64)
template <int MTH>
struct PRow {
  static constexpr int KF = MTH / 2, TAIL = MTH & 1;
  u16x8_t f[KF > 0 ? KF : 1];
  s16x4_t t;
};
template <int MTH>
INA_DEVICE void p_rows(const unsigned char* img, int q, int n, PRow<MTH>& P) {
  const int m = mask_p(n);
  const unsigned char* row = img + n * IMG_ROW;
#pragma unroll
  for (int kb = 0; kb < PRow<MTH>::KF; ++kb)
    P.f[kb] = *reinterpret_cast<const u16x8_t*>(row + (((8 * kb + 2 * q) ^ m) << 3));
  if (PRow<MTH>::TAIL) P.t = *reinterpret_cast<const s16x4_t*>(row + (((8 * PRow<MTH>::KF + q) ^ m) << 3));
}
// T^T[(s,c)][query 16 qt + n] = P_g Q_g^T
template <int MTH, int QT>
INA_DEVICE f32x4_t tt(const PRow<MTH>& P, const QFrag<MTH, QT>& Qf, int qt) {
  f32x4_t T = Z4;
#pragma unroll
  for (int kb = 0; kb < PRow<MTH>::KF; ++kb) T = mfma_bf16(P.f[kb], Qf.f[qt][kb], T);
  if (PRow<MTH>::TAIL) T = mfma_tail(P.t, Qf.t[qt], T);
  return T;
}

// ------------------------------------------------------------------------------------------
template <int MTH, int QT, int SG>
__global__ __launch_bounds__(NT_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void ntn_fwd_kernel(NtnArgs k) {
  constexpr int GM = QT <= 2 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char ntn_lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Geo g = geo(k, n);
  const int t0 = (int)((long)k.ntile * blockIdx.y / gridDim.y), t1 = (int)((long)k.ntile * (blockIdx.y + 1) / gridDim.y);
  unsigned char* const zero = ntn_lds + 2 * k.tpb;
  uint32_t woff = 2 * k.tpb + ZERO_BYTES + wave * (GM * PIMG);   // the wave's P images
  for (int i = lane; i < GM * PIMG / 16; i += 64) reinterpret_cast<u32x4_t*>(ntn_lds + woff)[i] = u32x4_t{0u, 0u, 0u, 0u};
  if (wave == 0)
    for (int i = lane; i < ZERO_BYTES / 16; i += 64) reinterpret_cast<u32x4_t*>(zero)[i] = u32x4_t{0u, 0u, 0u, 0u};
  const int nfrag = k.tpb >> 10;
  const unsigned char* tiles = reinterpret_cast<const unsigned char*>(k.tiles);
  constexpr int fo = SG * MTH * 16 * IMG_ROW;   // FC fragments after the M images
  for (int grp = blockIdx.x; grp * NW * g.G < k.E; grp += gridDim.x) {
    const int epw = (grp * NW + wave) * g.G;
    CFrag<MTH> Cf;
    load_cf<MTH>(k, g, epw, q, Cf);
    QFrag<MTH, QT> Qf[GM];
    f32x4_t Lg[GM][QT];
#pragma unroll
    for (int gi = 0; gi < GM; ++gi) {
      load_qf<MTH, QT>(k, g, epw + gi, gi < g.G && epw + gi < k.E, q, n, Qf[gi]);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) Lg[gi][qt] = Z4;
    }
    __syncthreads();   // the previous group's readers are done with the stage buffers
    stage_tile(ntn_lds, tiles + (long)t0 * k.tpb, nfrag);
    stage_wait();
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
      const unsigned char* buf = ntn_lds + ((t - t0) & 1) * k.tpb;
      if (t + 1 < t1) stage_tile(ntn_lds + ((t + 1 - t0) & 1) * k.tpb, tiles + (long)(t + 1) * k.tpb, nfrag);
      const int lt = opaque_lane(), q = lt >> 4, n = lt & 15;
      const Geo g = geo(k, n);
      p_images<MTH, SG>(buf, ntn_lds + woff, g, Cf, q, n);
      wave_order(woff);
      const s16x4_t wt = *reinterpret_cast<const s16x4_t*>(buf + fo + 512 + lt * 8);
#pragma unroll
      for (int gi = 0; gi < GM; ++gi) {
        if (gi < g.G) {
          PRow<MTH> Pa;
          p_rows<MTH>(ntn_lds + woff + gi * PIMG, q, n, Pa);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            const f32x4_t T = tt<MTH, QT>(Pa, Qf[gi], qt);   // rows (s, c), cols query
            Lg[gi][qt] = mfma16_bf16(wt, bf4relu(T), Lg[gi][qt]);
          }
        }
      }
      stage_wait();
      __syncthreads();
    }
#pragma unroll
    for (int gi = 0; gi < GM; ++gi) {
      const int ep = epw + gi;
      if (gi >= g.G || ep >= k.E) continue;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 4 * q + r, qi = 16 * qt + n;   // logits^T: rows class c', cols query
          if (c < g.N && qi < g.NQ) {
            const long o = ((long)ep * g.NQ + qi) * g.N + c;
            if (gridDim.y == 1)
              k.probs[o] = sigmoidf_(Lg[gi][qt][r] + k.bias[k.paper ? 0 : c]);
            else
              k.part[(long)blockIdx.y * k.E * g.NQ * g.N + o] = Lg[gi][qt][r];
          }
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
template <int MTH, int QT, int SG>
__global__ __launch_bounds__(NT_THREADS) __attribute__((amdgpu_waves_per_eu(2))) void ntn_bwd_kernel(NtnArgs k) {
  constexpr int GM = QT <= 2 ? 2 : 1;
  constexpr int KQ = (QT + 1) / 2;     // 32-deep K-steps over the queries
  constexpr int VIMG = KQ * 32 * 32;   // V / dT image [32 KQ rows (query)][16 cols (slice, class)] bf16
  constexpr int RA = 16 * MTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char ntn_lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15, wave = threadIdx.x >> 6;
  const Geo g = geo(k, n);
  const int t0 = (int)((long)k.ntile * blockIdx.y / gridDim.y), t1 = (int)((long)k.ntile * (blockIdx.y + 1) / gridDim.y);
  const bool split = gridDim.y > 1;
  unsigned char* const zero = ntn_lds + 2 * k.tpb;
  // the wave's images [P_0 .. P_{GM-1} | V | dT] at byte offset woff (laundered at every order point)
  uint32_t woff = 2 * k.tpb + ZERO_BYTES + wave * (GM * PIMG + 2 * VIMG);
  float* const dwl = reinterpret_cast<float*>(zero + ZERO_BYTES + NW * (GM * PIMG + 2 * VIMG));
  // zero once: rows / columns of the images no product writes (query rows >= 16 QT of V / dT, P columns >= H)
  for (int i = lane; i < (GM * PIMG + 2 * VIMG) / 16; i += 64)
    reinterpret_cast<u32x4_t*>(ntn_lds + woff)[i] = u32x4_t{0u, 0u, 0u, 0u};
  if (wave == 0)
    for (int i = lane; i < ZERO_BYTES / 16; i += 64) reinterpret_cast<u32x4_t*>(zero)[i] = u32x4_t{0u, 0u, 0u, 0u};
  const int nfrag = k.tpb >> 10;
  const unsigned char* tiles = reinterpret_cast<const unsigned char*>(k.tiles);
  constexpr int fo = SG * MTH * 16 * IMG_ROW;
  const float gs = k.gscale ? k.gscale[0] : 1.f;
  const int SGN = SG * g.N;
  const int dwe = k.paper ? SG : SGN * g.N;   // dw slab entries per tile
  const long hH = (long)k.h * g.H;
  unsigned short* const dp = reinterpret_cast<unsigned short*>(k.dp_out);
  unsigned short* const dp_trash = dp + ((long)k.E * g.N + 63) / 64 * 64 * hH;   // past the zero pad rows
  for (int grp = blockIdx.x; grp * NW * g.G < k.E; grp += gridDim.x) {
    const int epw = (grp * NW + wave) * g.G;
    CFrag<MTH> Cf;
    load_cf<MTH>(k, g, epw, q, Cf);
    if (k.cls_bf && !blockIdx.y && g.lrow && epw + g.lg < k.E) {
      unsigned short* crow = reinterpret_cast<unsigned short*>(k.cls_bf) + ((long)(epw + g.lg) * g.N + g.lc) * g.H;
#pragma unroll
      for (int ka = 0; ka < CFrag<MTH>::KF; ++ka) {
        const int a = 32 * ka + 8 * q;
        if (a < g.H) *reinterpret_cast<u16x8_t*>(crow + a) = Cf.f[ka];
      }
      if (CFrag<MTH>::TAIL) {
        const int a = 32 * CFrag<MTH>::KF + 4 * q;
        if (a < g.H) *reinterpret_cast<s16x4_t*>(crow + a) = Cf.t;
      }
    }
    QFrag<MTH, QT> Qf[GM];
    u16x8_t QB[GM][MTH][KQ];   // A = Q^T[i = b][k = query]
    s16x4_t dzT[GM][QT];       // B[k = c'][col = query] (16x16x16)
    u16x8_t dzB[GM][KQ];       // B[k = query][col = c']
    f32x4_t dQ[GM][MTH][QT];   // dQ^T[b][query]
#pragma unroll
    for (int gi = 0; gi < GM; ++gi) {
      const int ep = epw + gi;
      const bool oke = gi < g.G && ep < k.E;
      load_qf<MTH, QT>(k, g, ep, oke, q, n, Qf[gi]);
      const long rq0 = (long)(oke ? ep : 0) * (g.N * k.K + g.NQ) + g.N * k.K;
      const float* dze = k.dz + (long)(oke ? ep : 0) * g.NQ * g.N;
#pragma unroll
      for (int mb = 0; mb < MTH; ++mb)
#pragma unroll
        for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int b = 16 * mb + n, qi = 32 * kq + 8 * q + j;
            QB[gi][mb][kq][j] = f2bf(ldz(k.e, oke && qi < g.NQ && b < g.H, (rq0 + qi) * g.H + b));
          }
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qi = 16 * qt + n, cp = 4 * q + j;
          dzT[gi][qt][j] = (short)f2bf(gs * ldz(dze, oke && qi < g.NQ && cp < g.N, qi * g.N + cp));
        }
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int qi = 32 * kq + 8 * q + j;
          dzB[gi][kq][j] = f2bf(gs * ldz(dze, oke && qi < g.NQ && n < g.N, qi * g.N + n));
        }
#pragma unroll
      for (int mb = 0; mb < MTH; ++mb)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) dQ[gi][mb][qt] = Z4;
    }
    f32x4_t dC[MTH];   // dC^T[a][(g, c)]
#pragma unroll
    for (int ma = 0; ma < MTH; ++ma) dC[ma] = Z4;
    __syncthreads();
    stage_tile(ntn_lds, tiles + (long)t0 * k.tpb, nfrag);
    stage_wait();
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
      const int par = (t - t0) & 1;
      const unsigned char* buf = ntn_lds + par * k.tpb;
      if (t + 1 < t1) stage_tile(ntn_lds + (par ^ 1) * k.tpb, tiles + (long)(t + 1) * k.tpb, nfrag);
      const int lt = opaque_lane(), q = lt >> 4, n = lt & 15;
      const Geo g = geo(k, n);
      const int dsl = n / g.N, dcl = n - dsl * g.N;
      if (t > t0 && (int)threadIdx.x < dwe) {   // flush the previous tile's dw (slots complete: barrier)
        const float* src = dwl + (par ^ 1) * NW * DW_SLOT;
        float acc = 0.f;
        if (k.paper) {
          for (int w = 0; w < NW; ++w)
            for (int c = 0; c < g.N; ++c) acc += src[w * DW_SLOT + (threadIdx.x * g.N + c) * 16 + c];
        } else {
          const int row = threadIdx.x / g.N, cp = threadIdx.x - row * g.N;
          for (int w = 0; w < NW; ++w) acc += src[w * DW_SLOT + row * 16 + cp];
        }
        k.dw_slab[((long)grp * k.ntile + t - 1) * dwe + threadIdx.x] = acc;
      }
      p_images<MTH, SG>(buf, ntn_lds + woff, g, Cf, q, n);
      wave_order(woff);
      const s16x4_t wA = *reinterpret_cast<const s16x4_t*>(buf + fo + lt * 8);
      f32x4_t dw = Z4;
#pragma unroll
      for (int gi = 0; gi < GM; ++gi) {
        if (gi >= g.G) continue;
        const int ep = epw + gi;
        unsigned char* pg = ntn_lds + woff + gi * PIMG;
        unsigned char* vimg = ntn_lds + woff + GM * PIMG;
        unsigned char* dtimg = vimg + VIMG;
        PRow<MTH> Pa;
        p_rows<MTH>(pg, q, n, Pa);
        s16x4_t dT[QT];   // bf16 dT^T: rows (s, c), cols query (the dQ B operand and the dT image)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const f32x4_t T = tt<MTH, QT>(Pa, Qf[gi], qt);          // rows (s, c), cols query
          const f32x4_t dV = mfma16_bf16(wA, dzT[gi][qt], Z4);   // rows (s, c), cols query
          f32x4_t d;
#pragma unroll
          for (int r = 0; r < 4; ++r) d[r] = T[r] > 0.f ? dV[r] : 0.f;
          dT[qt] = bf4(d);
          // images [query row][(s, c) col]: the lane writes its query row's 4 (s, c) columns
          const int off = voff(16 * qt + n, q);
          *reinterpret_cast<s16x4_t*>(vimg + off) = bf4relu(T);
          *reinterpret_cast<s16x4_t*>(dtimg + off) = dT[qt];
        }
        wave_order(woff);
        pg = ntn_lds + woff + gi * PIMG;
        vimg = ntn_lds + woff + GM * PIMG;
        dtimg = vimg + VIMG;
        // transposed image reads: lane (q, n) gets image[32 kq + 8 q + j][col n], j < 8
        u16x8_t Vt[KQ], dTt[KQ];
#pragma unroll
        for (int kq = 0; kq < KQ; ++kq) {
          const int r0 = 32 * kq + 8 * q + (n >> 2);
          const int o0 = voff(r0, n & 3), o1 = voff(r0 + 4, n & 3);
          Vt[kq] = cat8(trr(vimg + o0), trr(vimg + o1));
          dTt[kq] = cat8(trr(dtimg + o0), trr(dtimg + o1));
        }
        // dw[(s, c)][c'] += sum_q V[(s, c), q] dz[q, c']
#pragma unroll
        for (int kq = 0; kq < KQ; ++kq) dw = mfma_bf16(Vt[kq], dzB[gi][kq], dw);
        // dQ^T[b][q] += sum_(s,c) P^T[b, (s,c)] dT^T[(s,c), q]   (A: the P image read transposed)
#pragma unroll
        for (int mb = 0; mb < MTH; ++mb) {
          const int pr = 4 * q + (n >> 2);
          const s16x4_t Pt = trr(pg + pr * IMG_ROW + (((4 * mb + (n & 3)) ^ mask_p(pr)) << 3));
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) dQ[gi][mb][qt] = mfma16_bf16(Pt, dT[qt], dQ[gi][mb][qt]);
        }
        // dP^T[b][(s, c)] = sum_q Q^T[b, q] dT[q, (s, c)]
        f32x4_t dPT[MTH];
#pragma unroll
        for (int mb = 0; mb < MTH; ++mb) {
          dPT[mb] = Z4;
#pragma unroll
          for (int kq = 0; kq < KQ; ++kq) dPT[mb] = mfma_bf16(QB[gi][mb][kq], dTt[kq], dPT[mb]);
        }
        // dP -> global bf16 [(e, c)][s H + b] (lanes outside the valid ranges store into the trash tail)
        {
          const int s = t * SG + dsl;
          const bool okc = n < SGN && s < k.h && ep < k.E;
          unsigned short* const drow = dp + ((long)(okc ? ep : 0) * g.N + dcl) * hH + (long)(okc ? s : 0) * g.H;
#pragma unroll
          for (int mb = 0; mb < MTH; ++mb) {
            const int b0 = 16 * mb + 4 * q;
            unsigned short* dst = (okc && b0 < g.H) ? drow + b0 : dp_trash;
            *reinterpret_cast<s16x4_t*>(dst) = bf4(dPT[mb]);
          }
        }
        wave_order(woff);   // this episode's P image reads are done: it becomes the dP image D[(s,c)][b]
        pg = ntn_lds + woff + gi * PIMG;
#pragma unroll
        for (int mb = 0; mb < MTH; ++mb)
          *reinterpret_cast<s16x4_t*>(pg + n * IMG_ROW + (((4 * mb + q) ^ mask_p(n)) << 3)) = bf4(dPT[mb]);
        wave_order(woff);   // (the next episode's V / dT image writes come after this one's reads)
      }
      wave_order(woff);
      const unsigned char* const pimg = ntn_lds + woff;
      // dC^T[a][(g, c)] += sum_b M_s[a, b] D_s[b, (g, c)], stacked over the wave's episodes (K over b: full
      // 32-deep steps + the 16-deep tail, as for P)
#pragma unroll
      for (int sl = 0; sl < SG; ++sl) {
        const unsigned char* mimg = buf + sl * (RA * IMG_ROW);
        const int row = sl * g.N + g.lc, mpr = mask_p(row);
        const unsigned char* drow = g.lrow ? pimg + g.lg * PIMG + row * IMG_ROW : zero;
        PRow<MTH> Bd;
#pragma unroll
        for (int kb = 0; kb < PRow<MTH>::KF; ++kb)
          Bd.f[kb] = *reinterpret_cast<const u16x8_t*>(g.lrow ? drow + (((8 * kb + 2 * q) ^ mpr) << 3) : zero);
        if (PRow<MTH>::TAIL)
          Bd.t = *reinterpret_cast<const s16x4_t*>(g.lrow ? drow + (((8 * PRow<MTH>::KF + q) ^ mpr) << 3) : zero);
#pragma unroll
        for (int ma = 0; ma < MTH; ++ma) {
          const int a = 16 * ma + n, mma = mask_m(a);
          const unsigned char* arow = mimg + a * IMG_ROW;
#pragma unroll
          for (int kb = 0; kb < PRow<MTH>::KF; ++kb)
            dC[ma] = mfma_bf16(*reinterpret_cast<const u16x8_t*>(arow + (((8 * kb + 2 * q) ^ mma) << 3)), Bd.f[kb], dC[ma]);
          if (PRow<MTH>::TAIL)
            dC[ma] = mfma_tail(*reinterpret_cast<const s16x4_t*>(arow + (((8 * PRow<MTH>::KF + q) ^ mma) << 3)), Bd.t,
                               dC[ma]);
        }
      }
      {   // this wave's dw tile -> its exchange slot (summed over the workgroup's waves after the barrier)
        float* slot = dwl + par * NW * DW_SLOT + wave * DW_SLOT;
#pragma unroll
        for (int r = 0; r < 4; ++r) slot[(4 * q + r) * 16 + n] = dw[r];
      }
      stage_wait();
      __syncthreads();
    }
    if (t1 > t0 && (int)threadIdx.x < dwe) {   // flush the last tile's dw
      const float* src = dwl + ((t1 - 1 - t0) & 1) * NW * DW_SLOT;
      float acc = 0.f;
      if (k.paper) {
        for (int w = 0; w < NW; ++w)
          for (int c = 0; c < g.N; ++c) acc += src[w * DW_SLOT + (threadIdx.x * g.N + c) * 16 + c];
      } else {
        const int row = threadIdx.x / g.N, cp = threadIdx.x - row * g.N;
        for (int w = 0; w < NW; ++w) acc += src[w * DW_SLOT + row * 16 + cp];
      }
      k.dw_slab[((long)grp * k.ntile + t1 - 1) * dwe + threadIdx.x] = acc;
    }
    // dC^T: rows a, col (g, c)
    {
      const int ep = epw + g.lg;
      if (g.lrow && ep < k.E) {
        float* dc_out = split ? k.part + (long)blockIdx.y * k.E * g.N * g.H : k.dcls;
#pragma unroll
        for (int ma = 0; ma < MTH; ++ma) {
          const int a0 = 16 * ma + 4 * q;
          if (a0 < g.H) *reinterpret_cast<f32x4_t*>(dc_out + ((long)ep * g.N + g.lc) * g.H + a0) = dC[ma];
        }
      }
    }
    // dQ^T: rows b, cols query -> the query rows of de (or this split's [E][NQ][H] partial)
#pragma unroll
    for (int gi = 0; gi < GM; ++gi) {
      const int ep = epw + gi;
      if (gi >= g.G || ep >= k.E) continue;
      const long rq0 = (long)ep * (g.N * k.K + g.NQ) + g.N * k.K;
      float* dq_base = split ? k.part2 + ((long)blockIdx.y * k.E + ep) * g.NQ * g.H : k.de + rq0 * g.H;
#pragma unroll
      for (int mb = 0; mb < MTH; ++mb)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const int b0 = 16 * mb + 4 * q, qi = 16 * qt + n;
          if (qi < g.NQ && b0 < g.H) *reinterpret_cast<f32x4_t*>(dq_base + (long)qi * g.H + b0) = dQ[gi][mb][qt];
        }
    }
    // (the next group's first barrier orders these dw-slot reads before its writes)
  }
}

// sums of the split partials, in split order (deterministic)
__global__ __launch_bounds__(256) void ntn_fwd_finish_kernel(const float* __restrict__ part, int ny, long n, int N,
                                                             int paper, const float* __restrict__ bias,
                                                             float* __restrict__ probs) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float s = 0.f;
    for (int y = 0; y < ny; ++y) s += part[(long)y * n + i];
    probs[i] = sigmoidf_(s + bias[paper ? 0 : (int)(i % N)]);
  }
}
__global__ __launch_bounds__(256) void ntn_bwd_finish_kernel(const float* __restrict__ pc, const float* __restrict__ pq,
                                                             int ny, int E, int N, int K, int Q, int H,
                                                             float* __restrict__ dcls, float* __restrict__ de) {
  const long n1 = (long)E * N * H, nqh = (long)N * Q * H, n2 = (long)E * nqh;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n1 + n2; i += (long)gridDim.x * 256) {
    float s = 0.f;
    if (i < n1) {
      for (int y = 0; y < ny; ++y) s += pc[(long)y * n1 + i];
      dcls[i] = s;
    } else {
      const long j = i - n1, ep = j / nqh, r = j - ep * nqh;
      for (int y = 0; y < ny; ++y) s += pq[(long)y * n2 + j];
      de[(ep * (long)(N * K + N * Q) + N * K) * H + r] = s;
    }
  }
}

int finish_grid(long n) {
  const long g = (n + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

int qt_of(int N, int Q) {
  const int need = (N * Q + 15) / 16;
  return need <= 1 ? 1 : (need <= 2 ? 2 : (need <= 4 ? 4 : 0));
}

size_t lds_bytes(const NtnArgs& a, int QT, bool bwd) {
  const int GM = QT <= 2 ? 2 : 1;
  const size_t per_wave = (size_t)GM * PIMG + (bwd ? 2 * ((QT + 1) / 2) * 32 * 32 : 0);
  return (size_t)2 * a.tpb + ZERO_BYTES + NW * per_wave + (bwd ? (size_t)2 * NW * DW_SLOT * 4 : 0);
}

template <int MTH, int QT, int SG, bool BWD>
int launch(const NtnArgs& a, hipStream_t st) {
  const int groups = ina::ntn_groups(a.E, a.N, a.Q);
  const int blocks = groups < a.blocks ? groups : a.blocks;
  const int ny = a.split > 1 ? a.split : 1;
  const size_t lds = lds_bytes(a, QT, BWD);
  const void* fn = BWD ? (const void*)ntn_bwd_kernel<MTH, QT, SG> : (const void*)ntn_fwd_kernel<MTH, QT, SG>;
  if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -1;
  if (BWD) {
    hipLaunchKernelGGL((ntn_bwd_kernel<MTH, QT, SG>), dim3(blocks, ny), dim3(NT_THREADS), lds, st, a);
  } else {
    hipLaunchKernelGGL((ntn_fwd_kernel<MTH, QT, SG>), dim3(blocks, ny), dim3(NT_THREADS), lds, st, a);
  }
  if (ny > 1) {
    if (BWD) {
      const long n = (long)a.E * a.N * a.H * (1 + a.Q);
      hipLaunchKernelGGL(ntn_bwd_finish_kernel, dim3(finish_grid(n)), dim3(256), 0, st, a.part, a.part2, ny, a.E, a.N,
                         a.K, a.Q, a.H, a.dcls, a.de);
    } else {
      const long n = (long)a.E * a.N * a.Q * a.N;
      hipLaunchKernelGGL(ntn_fwd_finish_kernel, dim3(finish_grid(n)), dim3(256), 0, st, a.part, ny, n, a.N, a.paper,
                         a.bias, a.probs);
    }
  }
  INA_CHECK_LAUNCH();
  return 0;
}

template <bool BWD>
int dispatch(const NtnArgs& a, hipStream_t st) {
  const int MTH = (a.H + 15) / 16, QT = qt_of(a.N, a.Q);
  if (a.N < 1 || a.N > 16 || QT == 0 || a.H % 8 != 0 || a.H > 64) return -1;
  if (a.SG != ina::ntn_slices_per_tile(a.N) || a.G != ina::ntn_episodes_per_wave(a.N, a.Q)) return -1;
  if (lds_bytes(a, QT, BWD) > 160 * 1024) return -1;
#define INA_NTN_SG(M, Q)                                  \
  if (a.SG == 1) return launch<M, Q, 1, BWD>(a, st);      \
  if (a.SG == 2) return launch<M, Q, 2, BWD>(a, st);      \
  if (a.SG == 3) return launch<M, Q, 3, BWD>(a, st);      \
  if (a.SG == 4) return launch<M, Q, 4, BWD>(a, st);
#define INA_NTN_QT(M)                   \
  if (QT == 1) { INA_NTN_SG(M, 1) }     \
  if (QT == 2) { INA_NTN_SG(M, 2) }     \
  if (QT == 4) { INA_NTN_SG(M, 4) }
  if (MTH == 1) { INA_NTN_QT(1) }
  if (MTH == 3) { INA_NTN_QT(3) }
  if (MTH == 4) { INA_NTN_QT(4) }
#undef INA_NTN_QT
#undef INA_NTN_SG
  return -1;
}

}  // namespace

// ------------------------------------------------------------------------------------------
namespace ina {

int ntn_slices_per_tile(int N) {
  const int s = 16 / (N > 0 ? N : 1);
  return s < 4 ? (s > 0 ? s : 1) : 4;
}
int ntn_episodes_per_wave(int N, int Q) {
  const int gm = qt_of(N, Q) <= 2 ? 2 : 1;
  const int s = 16 / (N > 0 ? N : 1);
  return s < gm ? (s > 0 ? s : 1) : gm;
}
int ntn_groups(int E, int N, int Q) {
  const int per = NW * ntn_episodes_per_wave(N, Q);
  return (E + per - 1) / per;
}
// tile-split factor for small episode batches: fill ~256 workgroups, >= 2 tiles per split
int ntn_split(int E, int N, int Q, int h) {
  const int groups = ntn_groups(E, N, Q), ntile = (h + ntn_slices_per_tile(N) - 1) / ntn_slices_per_tile(N);
  if (groups >= 64) return 1;
  int ny = 256 / groups;
  if (ny > ntile / 2) ny = ntile / 2;
  return ny > 1 ? ny : 1;
}
int ntn_fwd(const NtnArgs& a, hipStream_t st) { return dispatch<false>(a, st); }
int ntn_bwd(const NtnArgs& a, hipStream_t st) { return dispatch<true>(a, st); }

}  // namespace ina
