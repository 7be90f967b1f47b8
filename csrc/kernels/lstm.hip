// Persistent fused BiLSTM forward / BPTT backward for gfx950 (K1 + K2 + K3 + K11 of SURVEY 2.3).
//
// Reference semantics: TF BasicLSTMCell inside bidirectional_dynamic_rnn over ALL L steps
// (model/graph.py:34-49): gates = [x_t ; h_{t-1}] @ W + b, order i,j,f,o,
// c' = c*sig(f + 1) + sig(i)*tanh(j), h' = tanh(c')*sig(o).  x_t = [word_emb ; pos1_emb ; pos2_emb]
// gathered in-kernel (model/base.py:76-86).
//
// Layout ("lane ownership"): one wave owns 16 sequences of one direction.  Gates are computed
// transposed, G^T[4U, 16] = W^T[4U, K] x XH^T[K, 16], as U/4 M-tiles of v_mfma_f32_16x16x32_bf16
// (or v_mfma_f32_16x16x4_f32 in fp32 mode).  Row 16m + 4q + g of M-tile m is gate g of unit
// 4m + q, so the accumulator of lane (q = l>>4, n = l&15) holds i,j,f,o of unit 4m+q for sequence n
// in its 4 registers.  The K dimension is laid out so that lane group q supplies exactly the h
// units it owns (and x features 4xi+q): the recurrence h_t -> B operand never leaves the lane.
// The backward reuses the same trick for d[x;h] = W dG, and transposes (dG, XH) through
// wave-private LDS every 2 steps to accumulate dW with MFMAs (32 samples per K-step).
#include <type_traits>

#include <cstdlib>
#include "ina_common.h"
#include "ina_launch.h"


using namespace ina;


namespace {

template <int U, int NX, bool BF16>
struct Shape {
  static constexpr int U4 = U / 4;
  static constexpr int KPL = BF16 ? 8 : 1;                 // k values per lane per MFMA
  static constexpr int NSLOT = U4 + NX;                    // [h ; x] slots per lane group
  static constexpr int NKS = (NSLOT + KPL - 1) / KPL;      // fwd K-steps
  static constexpr int NMT = U4;                           // fwd M-tiles (16 gate rows each)
  static constexpr int NMT2 = (NSLOT + 3) / 4;             // bwd M-tiles over feature slots
  static constexpr int NG = 4 * U4;                        // gate slots per lane
  static constexpr int NKS2 = (NG + KPL - 1) / KPL;        // bwd K-steps over gate slots
  static constexpr int G4 = 4 * U;                         // gate columns
  static constexpr int GT = (G4 + 15) / 16;                // dW M-tiles (gate rows)
  static constexpr int KSTEP_SAMPLES = BF16 ? 32 : 4;      // samples per dW MFMA K-step
  static constexpr int RS = BF16 ? 40 : 36;                // LDS row stride (elements) for 32 samples
};

template <bool BF16>
struct FragT;
template <>
struct FragT<true> {
  using type = u16x8_t;
  using elem = unsigned short;
};
template <>
struct FragT<false> {
  using type = float;
  using elem = float;
};

template <bool BF16>
INA_DEVICE void fset(typename FragT<BF16>::type& fr, int j, float v);
template <>
INA_DEVICE void fset<true>(u16x8_t& fr, int j, float v) { fr[j] = f2bf(v); }
template <>
INA_DEVICE void fset<false>(float& fr, int, float v) { fr = v; }

template <bool BF16>
INA_DEVICE typename FragT<BF16>::type fzero();
template <>
INA_DEVICE u16x8_t fzero<true>() { return u16x8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
template <>
INA_DEVICE float fzero<false>() { return 0.f; }

INA_DEVICE f32x4_t mma(const u16x8_t& a, const u16x8_t& b, const f32x4_t& c) { return mfma_bf16(a, b, c); }
INA_DEVICE f32x4_t mma(float a, float b, const f32x4_t& c) { return mfma_f32(a, b, c); }

INA_DEVICE unsigned short to_elem(float v, unsigned short*) { return f2bf(v); }
INA_DEVICE float to_elem(float v, float*) { return v; }
INA_DEVICE float from_elem(unsigned short v) { return bf2f(v); }
INA_DEVICE float from_elem(float v) { return v; }

// Cell-state stash element: fp16 in bf16 mode (|c| <= L since |c_t - f c_{t-1}| < 1, far inside
// fp16 range; 11-bit mantissa), fp32 in the exact fp32 mode.
template <bool BF16>
struct CT {
  using type = float;
};
template <>
struct CT<true> {
  using type = _Float16;
};
INA_DEVICE float from_c(_Float16 v) { return (float)v; }
INA_DEVICE float from_c(float v) { return v; }

// lanes whose bit is set in the wave-uniform mask m take b, the others a (one v_cndmask with an
// SGPR-pair condition; the masks are ballots computed once per kernel).
INA_DEVICE uint32_t lane_sel(uint64_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}

// Per-lane source of x feature f = 4 xi + q (loop invariant): word / pos1 / pos2 table column, or
// none (f >= DIN).  The per-step gather is ONE unconditional load per feature: the row offset is
// picked with SGPR-mask selects (no lane-dependent branch around a load: hipcc would wait vmcnt(0)
// per element and serialise the L2 round trips).  "none" lanes load a finite word-table value that
// meets only zero weight rows (the packs are zero-padded past DIN) and is never staged for dW.
struct XSrc {
  const float* base;
  int col;
  int sel;               // 0 word, 1 pos1, 2 pos2, 3 none
  uint64_t mp1, mp2;     // wave-uniform lane masks
};
INA_DEVICE XSrc make_xsrc(int f, const float* __restrict__ wemb, int E, const float* __restrict__ p1emb,
                          const float* __restrict__ p2emb, int PD) {
  XSrc s;
  s.sel = f < E ? 0 : (f < E + PD ? 1 : (f < E + 2 * PD ? 2 : 3));
  s.base = s.sel == 1 ? p1emb : (s.sel == 2 ? p2emb : wemb);
  s.col = s.sel == 0 ? f : (s.sel == 1 ? f - E : (s.sel == 2 ? f - E - PD : 0));
  s.mp1 = __ballot(s.sel == 1);
  s.mp2 = __ballot(s.sel == 2);
  return s;
}
// element offsets of the step's token row in each table (24-bit multiplies: rows < 2^24 checked
// on the host)
struct XRow {
  uint32_t w, p1, p2;
};
INA_DEVICE XRow xrow(int wid, int p1, int p2, int E, int PD) {
  return XRow{(uint32_t)__umul24(wid, E), (uint32_t)__umul24(p1, PD), (uint32_t)__umul24(p2, PD)};
}
INA_DEVICE float gather_x(const XSrc& s, const XRow& r) {
  uint32_t off = lane_sel(s.mp1, r.w, r.p1);
  off = lane_sel(s.mp2, off, r.p2) + s.col;
  return s.base[off];
}

// exp2 range factor of gate type g (i, j, f, o): the kernels scale their gate weight rows and biases
// by it once (sigmoid_l2 / tanh_l2 in ina_common.h), and add the forget bias 1.0 to the f bias first.
// Weight fragment row = lane & 15, gate type = row & 3 = lane & 3 (csrc/kernels header comment).
INA_DEVICE float gate_scale(int g) { return g == 1 ? 2.f * LOG2E_F : LOG2E_F; }
INA_DEVICE float gate_bias(float b, int g) { return (b + (g == 2 ? 1.f : 0.f)) * gate_scale(g); }
INA_DEVICE u16x8_t fscale(u16x8_t a, float s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = f2bf(bf2f(a[j]) * s);
  return a;
}
INA_DEVICE float fscale(float a, float s) { return a * s; }

INA_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}


}  // namespace

// ------------------------------------------------------------------------------------------
// direct x (LstmArgs::xd; verdict r3 #6: x_gather's 485 MB xg record and its four re-reads per step go
// away).  The word features come from the per-token word rows (ops/encoder.py::word_rows, q-interleaved
// [f0 f4 f1 f5 f2 f6 f3 f7]: lane group q's two slots xi = 0, 1 are ONE dword at byte 4q of the token's
// 16-byte row; a sequence's rows are contiguous, so a 128-byte line serves 8 steps).  The position
// features come from block-resident LDS tables, since the ids are shifted aranges (pos = o_s + t):
//   T[(q * 2 + tb) * 2L + r][xi] = bf16 of feature 4 xi + q if it is a column of position table tb, row r
//                                  (else 0); padding sequences read rows 0.. and mask the result to 0
// A lane reads its two 8-byte entries at rows o1 + t / o2 + t and ORs them into the word dword: every slot
// is nonzero in at most one of the three sources, so the operand bits equal x_gather's.
// ------------------------------------------------------------------------------------------
__device__ inline void xd_build(unsigned short* T, int L, int E, int PD, const float* __restrict__ p1emb,
                                const float* __restrict__ p2emb) {
  const int R = 2 * L, N = 4 * 2 * R * 4;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const int xi = i & 3, r = (i >> 2) % R, qt = (i >> 2) / R, tb = qt & 1, q = qt >> 1;
    const int c = 4 * xi + q - E - tb * PD;
    float v = 0.f;
    if (r < 2 * L && c >= 0 && c < PD) v = (tb ? p2emb : p1emb)[r * PD + c];
    T[i] = f2bf(v);
  }
}
// a block's copy of the tables (built once per forward by x_gather block (0, 0) into global memory: building
// them in every recurrence block cost ~50 us of lstm_fwd prologue at 12,800 blocks); 16-byte chunks
__device__ inline void xd_copy(void* lds, const unsigned short* __restrict__ g, int L) {
  const uint4* s = reinterpret_cast<const uint4*>(g);
  uint4* d = reinterpret_cast<uint4*>(lds);
  for (int i = threadIdx.x; i < 8 * L; i += blockDim.x) d[i] = s[i];   // 4 * 2 * 2L * 4 * 2 bytes / 16
}

// direct x without dropout (eval / keep_prob = 1): x_gather has nothing left but the recurrences' position
// tables and pos_shift_gemm's t = 0 ids -- one thread per sequence instead of one per token (the full
// gather grid was ~100 us of block launches for an eval step of 16,384 episodes)
__global__ __launch_bounds__(256) void xd_ids_kernel(const int* __restrict__ inst, int S, const int* __restrict__ pos1,
                                                     const int* __restrict__ pos2, int L, int E, int PD,
                                                     const float* __restrict__ p1emb, const float* __restrict__ p2emb,
                                                     unsigned short* __restrict__ posb, unsigned short* __restrict__ xdtab) {
  if (blockIdx.x == 0) xd_build(xdtab, L, E, PD, p1emb, p2emb);
  const int seq = blockIdx.x * 256 + threadIdx.x;
  if (seq >= ((S + 15) / 16) * 16) return;   // (padding rows of the last tile: the clamped row, as x_gather)
  const long r = (long)inst[seq < S ? seq : S - 1] * L;
  posb[(size_t)(seq >> 4) * L * 16 + (seq & 15)] = (unsigned short)(pos1[r] | (pos2[r] << 8));
}

// ------------------------------------------------------------------------------------------
// encoder input gather (bf16 mode; K1 of SURVEY 2.3).  The recurrences used to gather their x
// features per step (a random 20-byte word-table row per token, 2 directions x fwd + bwd = 4 times
// per token, one step of prefetch): latency-bound on L2/MALL misses (kbench: 0.44 -> 0.29 ms
// forward without the gathers).  This kernel gathers every token ONCE with full memory-level
// parallelism (one thread per token) into the lane-ownership layout the recurrences consume as
// one coalesced 8-byte load per lane-step:
//   xg[tile][t][lane = 16 q + n][xi] = bf16 x feature 4 xi + q of sequence 16 tile + n at step t
//                                      (0 past DIN and for padding sequences >= S)
//   posb[tile][t][n] = pos1 | pos2 << 8 (position ids of the pos-table gradient kernels)
//   dmask[tile][dir][t][lane] = DropoutWrapper keep bits (bit m: unit 4m + q), when dropout is on --
//                                the counter hash of lstm_fwd's fp32 path, off the recurrence's
//                                critical path (it was ~1/3 of the bf16 forward's VALU per step)
// x enters the gate MFMAs as bf16 in this mode, so the values are exactly the ones the per-step
// gather produced.
// ------------------------------------------------------------------------------------------
// a_lo = 2 a_lo + (x[15:0] < thr16), a_hi = 2 a_hi + (x[31:16] < thr16): an SDWA compare into VCC and an
// add-with-carry per bit (hipcc emits compare, select and or)
INA_DEVICE void keep_acc2(uint32_t x, uint32_t thr16, uint32_t& a_lo, uint32_t& a_hi) {
  asm("v_cmp_lt_u32_sdwa vcc, %2, %3 src0_sel:WORD_0 src1_sel:DWORD\n\t"
      "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc\n\t"
      "v_cmp_lt_u32_sdwa vcc, %2, %3 src0_sel:WORD_1 src1_sel:DWORD\n\t"
      "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
      : "+v"(a_lo), "+v"(a_hi)
      : "v"(x), "s"(thr16)
      : "vcc");
}
constexpr int XG_T = 16;   // steps per workgroup pass (16 sequences x 16 steps = 256 threads)
constexpr int XG_C = 3;    // passes per workgroup (L = 37: one workgroup per tile): the token loads of all
                           // passes are issued before any is consumed, the pos tables staged once
// UT / ET / PT: compile-time U, word dim and position dim (0 = the runtime arguments): the reference
// default (U 20, 5-d words, 5-d positions) gets a fully unrolled, branch-free feature select and keep-bit
// hash loop
template <int NX, bool DIRECT, int UT = 0, int ET = 0, int PT = 0>
__global__ __launch_bounds__(256) void x_gather_kernel(const int* __restrict__ inst, int S,
                                                      const int* __restrict__ word, const int* __restrict__ pos1,
                                                      const int* __restrict__ pos2, int L,
                                                      const float* __restrict__ wemb,
                                                      const unsigned short* __restrict__ wrows, int E,
                                                      const float* __restrict__ p1emb,
                                                      const float* __restrict__ p2emb, int PD,
                                                      unsigned short* __restrict__ xg,
                                                      unsigned short* __restrict__ posb,
                                                      unsigned char* __restrict__ dmask, int U, uint32_t seed,
                                                      const int* __restrict__ seed_dev, uint32_t thr,
                                                      const int* __restrict__ perm, unsigned short* __restrict__ xdtab,
                                                      const int* __restrict__ tlen) {
  // direct x: block (0, 0) also builds the recurrences' position tables (xd_build) in global memory
  if (xdtab != nullptr && blockIdx.x == 0 && blockIdx.y == 0) xd_build(xdtab, L, E, PD, p1emb, p2emb);
  // the two position tables ([2L, PD] each, tiny) in LDS: per-feature loads from them were most of
  // this kernel's vector-memory instructions
  __shared__ float ptab[2 * 128 * 8];
  __shared__ uint32_t kst[2 * XG_C * XG_T * 16];   // keep bytes [dir][step - t0][64 lanes]
  const int t0 = blockIdx.y * XG_C * XG_T;
  if constexpr (UT > 0) U = UT;
  if constexpr (ET > 0) E = ET;
  if constexpr (PT > 0) PD = PT;
  const int PTN = 2 * L * PD;
  // thread = one token (sequence n = tid & 15, step t0 + tid / 16): its id / row loads are runs along
  // t (coalesced), and it writes its NX x 4 features as 4 lane-group chunks; for a fixed step the
  // 16 sequences' chunks of one lane group are one contiguous 16 x 8-byte segment.
  const int ntiles = (S + 15) / 16;
  // grid-stride over tiles (the launcher may cap the grid: fewer, longer-lived workgroups)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int n = threadIdx.x & 15;
  const int seq = tile * 16 + n;
  const bool valid = seq < S;
  const long rb = (long)inst[valid ? seq : S - 1] * L;
  // dropout hash inputs, loaded once (inside the pass / direction loops they were 6 dependent load round
  // trips per thread): the counter uses the row's ORIGINAL index (ragged tiles sort the rows), so the mask
  // equals the unsorted run's and the oracle's
  const uint32_t sd = seed_dev ? (uint32_t)seed_dev[0] : seed;
  const uint32_t pv = perm ? (uint32_t)perm[valid ? seq : S - 1] : 0u;   // (clamped: no lane-dependent branch)
  const uint32_t oseq = (perm && valid) ? pv : (uint32_t)seq;
  // ragged tiles: keep bits of steps t >= the tile's longest length are never consumed (the attention stops
  // there and lstm_bwd's dH loads past it return 0): not hashed, stored as 0 (~30% of the hashes at FewRel lengths)
  const int Lhash = tlen ? tlen[tile] : L;
  int p1c[XG_C], p2c[XG_C], widc[XG_C];
  u16x8_t wrc[XG_C];
  // direct x: only the t = 0 position ids are consumed (pos_shift_gemm's per-sequence offsets); every
  // thread loads its sequence's first ids (16 distinct rows per wave) and no x features are written
  const bool xd = xg == nullptr;
#pragma unroll
  for (int c = 0; c < XG_C; ++c) {   // clamped rows: unconditional loads
    const int t = (blockIdx.y * XG_C + c) * XG_T + (threadIdx.x >> 4);
    const long r = rb + (xd ? 0 : min(t, L - 1));
    p1c[c] = pos1[r];
    p2c[c] = pos2[r];
    // DIRECT: the token's word row as one 16-byte load of 8 bf16 (E <= 8, zero padded, q-interleaved:
    // feature f at 2 (f & 3) + (f >> 2)).  xg == nullptr (direct-x recurrences): ids / keep bits only
    if (xd) continue;
    if constexpr (DIRECT) wrc[c] = *reinterpret_cast<const u16x8_t*>(wrows + r * 8);
    else widc[c] = word[r];
  }
  // (the pos tables are staged while those loads are in flight)
  if (!xd) {
    for (int i = threadIdx.x; i < 2 * PTN; i += 256) ptab[i] = i < PTN ? p1emb[i] : p2emb[i - PTN];
    __syncthreads();
  }
  const int DIN = E + 2 * PD;
#pragma unroll
  for (int c = 0; c < XG_C; ++c) {
  const int t = (blockIdx.y * XG_C + c) * XG_T + (threadIdx.x >> 4);
  if (t >= L) break;   // t grows with c
  const int p1 = p1c[c], p2 = p2c[c];
  if (xg != nullptr) {   // uniform
  const float* p1row = ptab + p1 * PD;
  const float* p2row = ptab + PTN + p2 * PD;
  u16x8_t wr = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (DIRECT) wr = wrc[c];
  const float* wrow = wemb + (DIRECT ? 0 : (long)widc[c] * E);
  float x[4 * NX];
#pragma unroll
  for (int f = 0; f < 4 * NX; ++f) {   // E, PD are kernel arguments: the source branches are uniform
    float wv = 0.f;
    if (f < E) wv = DIRECT ? bf2f(wr[f < 8 ? 2 * (f & 3) + (f >> 2) : 0]) : wrow[f];
    x[f] = f < E ? wv : (f < E + PD ? p1row[f - E] : (f < DIN ? p2row[f - E - PD] : 0.f));
  }
  unsigned short* dst = xg + (size_t)(tile * L + t) * 64 * NX;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned short v[NX];
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) v[xi] = f2bf(valid ? x[4 * xi + q] : 0.f);
#pragma unroll
    for (int c = 0; c < NX / 4; ++c)
      *reinterpret_cast<u16x4_t*>(dst + (q * 16 + n) * NX + 4 * c) =
          u16x4_t{v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
  }
  }
  if (!xd || t == 0) posb[(size_t)(tile * L + t) * 16 + n] = (unsigned short)(p1 | (p2 << 8));
  if (dmask) {   // uniform
    const uint32_t thr16 = thr >> 16;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const uint32_t salt = dropout_salt(sd, (uint32_t)d);
      const uint32_t pbase = ((oseq * L + t) * U) >> 1;   // U even: the row's first unit pair
      uint32_t by[4] = {0u, 0u, 0u, 0u};                            // keep byte of lane group q
      if (t < Lhash) {
        // dropout_mix(salt, pbase + k) with the counter multiply strength-reduced (salt folded into the row's
        // base), and the keep bits shift-accumulated (compare + add-with-carry per bit): unit 2k goes to byte
        // (2k) & 3 at bit k >> 1, so walking k DOWN leaves each bit at its place (lstm_keep's bits exactly)
        uint32_t b0 = pbase * 0x6C8E9CF5u + salt;
        asm volatile("" : "+v"(b0));   // one add per hash below (hipcc re-split it into base + k C1, then + salt)
#pragma unroll
        for (int k = 15; k >= 0; --k) {                             // units 2k, 2k + 1 (lstm_keep)
          if (2 * k >= U) continue;
          uint32_t x = b0 + (uint32_t)k * 0x6C8E9CF5u;
          x ^= x >> 16;
          x *= 0x7FEB352Du;
          x ^= x >> 15;
          const int g = (2 * k) & 3;
          keep_acc2(x, thr16, by[g], by[g + 1]);
        }
      }
      // staged in LDS, stored below as coalesced dwords (per-lane byte stores to global were most of
      // this kernel's time once direct x removed its x rows)
      unsigned char* mrow = reinterpret_cast<unsigned char*>(kst) + (d * XG_C * XG_T + t - t0) * 64 + n;
#pragma unroll
      for (int q = 0; q < 4; ++q) mrow[16 * q] = (unsigned char)by[q];
    }
  }
  }
  if (dmask) {   // uniform: the block's keep bytes, rows [t0, t0 + rows) of both directions
    __syncthreads();
    const int rows = min(XG_C * XG_T, L - t0), nw = rows * 16;
    for (int i = threadIdx.x; i < 2 * nw; i += 256) {
      const int d = i >= nw ? 1 : 0, r = i - d * nw;
      reinterpret_cast<uint32_t*>(dmask + (size_t)((tile * 2 + d) * L + t0) * 64)[r] = kst[d * XG_C * XG_T * 16 + r];
    }
    __syncthreads();   // kst is rewritten by the next tile
  }
  }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// DROP / STORE are compile-time so the step loop has no branches: the waitcnt pass can then count
// the stores issued after each prefetch and wait only for the prefetched loads.
// SKIP (bf16): sequence_length semantics for the backward direction (lstm_skip_padding): it starts at the
// tile's longest length and each row's state is reset to zero past its own length (TF dynamic_rnn)
#ifndef INA_FWD_WAVES
#define INA_FWD_WAVES 5   // bf16 waves per SIMD (the gate fragments in LDS free the registers)
#endif
template <int U, int NX, bool BF16, bool DROP, bool STORE, bool SKIP = false, bool XD = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BF16 && U <= 20 ? INA_FWD_WAVES : 4))) void lstm_fwd_kernel(
    const int* __restrict__ inst, int S, const int* __restrict__ word, const int* __restrict__ pos1,
    const int* __restrict__ pos2, int L, const float* __restrict__ wemb, int E,
    const float* __restrict__ p1emb, const float* __restrict__ p2emb, int PD,
    const typename FragT<BF16>::type* __restrict__ apack, const float* __restrict__ bias,
    typename FragT<BF16>::elem* __restrict__ hlane, typename CT<BF16>::type* __restrict__ cst,
    typename FragT<BF16>::elem* __restrict__ hnat, unsigned char* __restrict__ dmask, uint32_t seed, uint32_t thr,
    float inv_kp, int drop, const int* __restrict__ seed_dev, const unsigned short* __restrict__ xg,
    const int* __restrict__ tlen, const int* __restrict__ slen, const unsigned short* __restrict__ wrows,
    uint32_t wbytes) {
  static_assert(!XD || (BF16 && NX == 4), "direct x: bf16, 4 x slots per lane");
  if (seed_dev) seed = (uint32_t)seed_dev[0];   // device-resident dropout seed (HIP-graph replay)
  using Sh = Shape<U, NX, BF16>;
  using frag = typename FragT<BF16>::type;
  using celem = typename CT<BF16>::type;
  constexpr int U4 = Sh::U4, KPL = Sh::KPL, NKS = Sh::NKS, NMT = Sh::NMT;
  extern __shared__ __attribute__((aligned(16))) int2 ids_all[];
  // wave index as an SGPR: the tile, its step count and every per-step record / x address derive from it, and as a
  // VGPR each step paid a v_mul_lo_u32 + 64-bit address add for the record stores and the loop counters on the VALU
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, n = lane & 15;
  // longest work first: the backward direction (all L steps) dispatches before the forward one, whose ragged tiles
  // (length-sorted ascending by the plan) run longest first -- no long tile left for the kernel's tail (lstm_fwd
  // 784 -> 772, lstm_bwd 1343 -> 1322, rec_attn_fwd 365 -> 354 us, same box: profiles/r6_lpt)
  const int dir = 1 - (int)blockIdx.y;
  const int ntiles = (S + 15) / 16;
  const int tile = dir == 0 ? ntiles - 1 - ((int)blockIdx.x * 4 + wave) : (int)blockIdx.x * 4 + wave;
  int2* ids = ids_all + (wave * 16) * L;
  // bf16: the direction's gate weight fragments (pre-scaled) live in LDS and are read per step instead of held in
  // 4 * NMT * NKS VGPRs per lane -- the registers that let a 5th wave per SIMD fit (u = 20: 128 -> 82 VGPRs,
  // kernel 732 -> 703 us; 6 waves spill in the step loop and measure 707: profiles/r6_flds)
  __shared__ frag lA[BF16 ? NMT * NKS * 64 : 1];
  const frag* ap = apack + (size_t)dir * NMT * NKS * 64;
  if constexpr (BF16) {
    for (int i = threadIdx.x; i < NMT * NKS * 64; i += 256) lA[i] = fscale(ap[i], gate_scale(i & 3));
  }
  if constexpr (XD) xd_copy(ids_all, xg, L);   // the block's position tables (xg = x_gather's global copy)
  if constexpr (BF16 || XD) __syncthreads();   // (before any wave leaves)
  constexpr bool FG = !BF16;   // fp32 mode gathers x per step
  if constexpr (FG) {
    // fp32 mode gathers x per step: stage (word, pos1 | pos2 << 16) of the wave's 16 sequences into LDS
    for (int i = lane; i < 16 * L; i += 64) {
      int sn = i / L, t = i - sn * L;
      int sq = tile * 16 + sn;
      int2 v = make_int2(0, 0);
      if (tile >= 0 && tile < ntiles && sq < S) {
        long r = (long)inst[sq] * L + t;
        v.x = word[r];
        v.y = pos1[r] | (pos2[r] << 16);
      }
      ids[i] = v;
    }
    wave_lds_sync();
  }
  if (tile < 0 || tile >= ntiles) return;
  const int seq = tile * 16 + n;  // rows >= S are padding rows of hnat (allocated to 16 * ntiles)
  const uint32_t salt = dropout_salt(seed, (uint32_t)dir);
  // ragged tiles: processing steps [tb, te).  Forward direction: t < Lt (the tile's longest length; later
  // outputs are masked out of the attention and its final state is unused).  Backward direction: all L
  // (parity: it runs through the padding first), or t < Lt with per-row resets (SKIP).
  const int Lt = tlen ? tlen[tile] : L;
  const int tb = (SKIP && dir == 1) ? L - Lt : 0, te = dir == 0 ? Lt : L;
  const int mylen = SKIP ? (seq < S ? slen[seq] : 0) : L;

  frag A[NMT][NKS];   // fp32: the fragments in registers
  if constexpr (!BF16) {
#pragma unroll
    for (int m = 0; m < NMT; ++m)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) A[m][ks] = fscale(ap[(m * NKS + ks) * 64 + lane], gate_scale(lane & 3));
  }
  float bm[NMT][4];   // pre-scaled gate biases (gate_bias)
#pragma unroll
  for (int m = 0; m < NMT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) bm[m][r] = gate_bias(bias[dir * 4 * U + r * U + 4 * m + q], r);

  float h[U4], c[U4];
#pragma unroll
  for (int m = 0; m < U4; ++m) h[m] = c[m] = 0.f;

  XSrc xs[NX];
#pragma unroll
  for (int xi = 0; xi < NX; ++xi) xs[xi] = make_xsrc(4 * xi + q, wemb, E, p1emb, p2emb, PD);
  int pofs[NX];   // lane's element offset inside a dxp [NPF][16] step block (pos features only)
#pragma unroll
  for (int xi = 0; xi < NX; ++xi) pofs[xi] = (4 * xi + q - E) * 16 + n;
  auto load_x = [&](int t, float* xv) {
    if constexpr (!FG) {   // x_gather_kernel output: one coalesced 8-byte load per 4 features
      const unsigned short* xp = xg + ((uint32_t)(tile * L + t) * 64 + lane) * NX;
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) {
        const u16x4_t v = *reinterpret_cast<const u16x4_t*>(xp + 4 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[4 * c + e] = bf2f(v[e]);
      }
    } else {
      const int2 id = ids[n * L + t];
      const XRow r = xrow(id.x, id.y & 0xffff, id.y >> 16, E, PD);
#pragma unroll
      for (int xi = 0; xi < NX; ++xi) xv[xi] = gather_x(xs[xi], r);
    }
  };
  // bf16: the recurrent h as packed bf16 pairs (units 2k, 2k + 1) -- the value the gate MFMA, the step record and
  // the next step read, converted ONCE per pair.  (h kept in fp32 rounded to bf16 cost a convert + a shift per
  // unit and step, and the B operand and the record store converted it again; x went bf16 -> fp32 -> bf16.)
  constexpr int NHW = (U4 + 1) / 2;
  uint32_t hw[NHW];
#pragma unroll
  for (int k = 0; k < NHW; ++k) hw[k] = 0u;
  // B operand word of slots (s0, s0 + 1): slot s < U4 is h unit s, U4 <= s < U4 + NX the x feature slot s - U4
  // (xw: NX / 2 words of packed bf16 pairs), past them zero.  Same-word aligned pairs pass through, the rest is one
  // v_perm (bytes 0-3 of src1 = the lo word, 4-7 of src0 = the hi word).
  auto bword = [&](const int s0, const uint32_t* xw) __attribute__((always_inline)) -> uint32_t {
    // source of slot s: word id (h word k -> k, x word k -> NHW + k, none -> -1) and 16-bit half
    auto wid = [&](int s) { return s < U4 ? (s >> 1) : (s - U4 < NX ? NHW + ((s - U4) >> 1) : -1); };
    auto half = [&](int s) { return s < U4 ? (s & 1) : ((s - U4) & 1); };
    auto word = [&](int id) { return id < NHW ? hw[id] : xw[id - NHW]; };
    const int il = wid(s0), ih = wid(s0 + 1), lh = half(s0), hh = half(s0 + 1);
    if (il < 0 && ih < 0) return 0u;
    if (il == ih && lh == 0 && hh == 1) return word(il);
    const uint32_t sl = il >= 0 ? (uint32_t)((2 * lh) | ((2 * lh + 1) << 8)) : 0x0C0Cu;
    const uint32_t sh = ih >= 0 ? (uint32_t)((4 + 2 * hh) | ((5 + 2 * hh) << 8)) : 0x0C0Cu;
    return __builtin_amdgcn_perm(ih >= 0 ? word(ih) : 0u, il >= 0 ? word(il) : 0u, sl | (sh << 16));
  };
  auto pk2 = [](float a, float b) {   // two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32, RNE as f2bf)
    typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
    const bf2_t v = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, v);
  };
  // one bf16 recurrence step at processing index tau with input feature words xw
  auto step_bf = [&](const int tau, const uint32_t* xw) __attribute__((always_inline)) {
    const int t = dir ? (L - 1 - tau) : tau;
    frag B[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if constexpr (BF16) {
        const u32x4_t v = {bword(ks * 8, xw), bword(ks * 8 + 2, xw), bword(ks * 8 + 4, xw), bword(ks * 8 + 6, xw)};
        B[ks] = __builtin_bit_cast(frag, v);
      }
    }
    float hv[U4];
#pragma unroll
    for (int m = 0; m < NMT; ++m) {
      f32x4_t acc = {bm[m][0], bm[m][1], bm[m][2], bm[m][3]};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) acc = mma(lA[(m * NKS + ks) * 64 + lane], B[ks], acc);
      // c[m] holds the cell state times 2 log2(e) (tanh_l2's argument scale): the scale rides on the g gate's
      // 1 - 2r form (k - 2k r, same fma) and the fp16 record's conversion (x 1/k), so tanh(c) needs no multiply
      const float ig = sigmoid_l2(acc[0]), fg = sigmoid_l2(acc[2]), og = sigmoid_l2(acc[3]);
      const float jk = fmaf(fast_rcp(__builtin_amdgcn_exp2f(acc[1]) + 1.0f), -2.f * (2.f * LOG2E_F), 2.f * LOG2E_F);
      c[m] = c[m] * fg + ig * jk;
      hv[m] = tanh_l2(c[m]) * og;
    }
    if constexpr (SKIP) {   // backward direction past the row's length: state (and output) reset to zero
      if (dir == 1 && t >= mylen) {
#pragma unroll
        for (int m = 0; m < U4; ++m) hv[m] = c[m] = 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < NHW; ++k) hw[k] = pk2(hv[2 * k], 2 * k + 1 < U4 ? hv[2 * k + 1] : 0.f);
    // bf16 step record [tile][dir][t][2][U4][64] (16-bit): slot 0 = the raw recurrent h (bf16), slot 1 = the cell
    // state (fp16, training only); every store is a coalesced 128-B lane-layout run off ONE address.  The h slot is
    // both the backward's stash and the attention input (the attention applies the DropoutWrapper mask from the keep
    // bits).  32-bit offsets (checked on the host); padding rows are stored too.
    unsigned short* rec = reinterpret_cast<unsigned short*>(hnat) + ((uint32_t)((tile * 2 + dir) * L + t) * (2 * U4)) * 64 + lane;
#pragma unroll
    for (int m = 0; m < U4; ++m) rec[m * 64] = (unsigned short)(hw[m >> 1] >> (16 * (m & 1)));
    if constexpr (STORE) {
#pragma unroll
      for (int m = 0; m < U4; ++m)
        rec[(U4 + m) * 64] = __builtin_bit_cast(unsigned short, (_Float16)(c[m] * (0.5f / LOG2E_F)));
    }
    if constexpr (DROP) {
      const uint32_t base = ((uint32_t)seq * L + t) * U + q;
      uint32_t bits = 0;
#pragma unroll
      for (int m = 0; m < U4; ++m) bits |= lstm_keep(salt, base + 4 * m, thr) ? (1u << m) : 0u;
      dmask[(uint32_t)((tile * 2 + dir) * L + t) * 64 + lane] = (unsigned char)bits;
    }
  };
  // one fp32 recurrence step at processing index tau with input features xv
  auto step = [&](const int tau, const float* xv) __attribute__((always_inline)) {
    const int t = dir ? (L - 1 - tau) : tau;
    frag B[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      B[ks] = fzero<BF16>();
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const int idx = ks * KPL + j;
        if (idx < U4)
          fset<BF16>(B[ks], j, h[idx]);
        else if (idx - U4 < NX)
          fset<BF16>(B[ks], j, xv[idx - U4]);
      }
    }
#pragma unroll
    for (int m = 0; m < NMT; ++m) {
      f32x4_t acc = {bm[m][0], bm[m][1], bm[m][2], bm[m][3]};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) acc = mma(A[m][ks], B[ks], acc);
      const float ig = sigmoid_l2(acc[0]), jg = tanh_l2(acc[1]), fg = sigmoid_l2(acc[2]), og = sigmoid_l2(acc[3]);
      c[m] = c[m] * fg + ig * jg;
      h[m] = tanh_l2(c[m] * (2.f * LOG2E_F)) * og;
    }
    if constexpr (SKIP) {   // backward direction past the row's length: state (and output) reset to zero
      if (dir == 1 && t >= mylen) {
#pragma unroll
        for (int m = 0; m < U4; ++m) h[m] = c[m] = 0.f;
      }
    }
    if constexpr (!BF16) {
      // fp32: the attention input (dropout applied) in natural rows, h / c stash in the lane layout
      typename FragT<BF16>::elem* hn = hnat + (((uint32_t)seq * L + t) * (2 * U) + dir * U + q);
      if constexpr (DROP) {
        const uint32_t base = ((uint32_t)seq * L + t) * U + q;
        uint32_t bits = 0;
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          const bool keep = lstm_keep(salt, base + 4 * m, thr);
          bits |= keep ? (1u << m) : 0u;
          hn[4 * m] = to_elem(keep ? h[m] * inv_kp : 0.f, (typename FragT<BF16>::elem*)nullptr);
        }
        if constexpr (STORE) {   // the backward re-applies the mask from these bits (no re-hashing)
          if constexpr (U4 <= 8) dmask[(uint32_t)((tile * 2 + dir) * L + t) * 64 + lane] = (unsigned char)bits;
        }
      } else {
#pragma unroll
        for (int m = 0; m < U4; ++m) hn[4 * m] = to_elem(h[m], (typename FragT<BF16>::elem*)nullptr);
      }
      if constexpr (STORE) {
        typename FragT<BF16>::elem* hp = hlane + ((uint32_t)((tile * 2 + dir) * L + t) * U4) * 64 + lane;
#pragma unroll
        for (int m = 0; m < U4; ++m) hp[m * 64] = to_elem(h[m], (typename FragT<BF16>::elem*)nullptr);
        celem* cp = cst + ((uint32_t)((tile * 2 + dir) * L + t) * U4) * 64 + lane;
#pragma unroll
        for (int m = 0; m < U4; ++m) cp[m * 64] = (celem)c[m];
      }
    }
  };
  // two-step unrolled loop with ping-pong x buffers: the gather for step tau+1 is issued before
  // step tau's math and consumed one step later (no register copies).  The loop body is ONE basic
  // block (odd-L tail peeled, prefetch index clamped) so LLVM cannot sink the prefetch loads down
  // to their uses.
  auto tof = [&](int tau) { return dir ? (L - 1 - tau) : tau; };
  // (Round 1 streamed the bf16 x rows through an inline-asm load ring retired by hand-counted
  // `s_waitcnt vmcnt(n)` waits.  It was removed: at u=8 it returned stale x values in 8 of 12
  // back-to-back runs (tools/dbg/u8_repro2.py; profiles/r2_v2), i.e. the count of VMEM ops retiring
  // after a load is not a safe completion bound, and an inline-asm load destination is invisible to
  // the register allocator (a spilled / copied in-flight destination corrupts state).  The loads
  // below are compiler-visible; the waitcnt pass inserts the waits.)
  // bf16: the ping-pong buffers hold the RAW x_gather rows, converted inside the step: converting at
  // the load made the compiler wait for it right there (s_waitcnt vmcnt(0), which also drained the
  // previous step's record stores), i.e. no prefetch at all
  if constexpr (XD) {
    // direct x: per step one dword of the token's word row (buffer load; padding sequences read past the
    // range -> 0) and two 8-byte LDS table entries, prefetched one step ahead like the xg rows below.
    // (The word loads two steps ahead, a 4-step loop, measured equal: 765 vs 768 us, profiles/r4_direct_x/pf2;
    // the tables read from x_gather's global copy through L1 instead of LDS, slower: 793 vs 766 us, gtab/.)
    const bool valid = seq < S;
    const int rb0 = inst[valid ? seq : S - 1] * L;
    const uint32_t wvo = valid ? (uint32_t)rb0 * 16u + 4u * (uint32_t)q : 0x80000000u;
    const int R = 2 * L;
    const uint32_t vm = valid ? 0xFFFFFFFFu : 0u;   // padding sequences: x = 0
    // (the table reads are 47% LDS bank conflicts -- 16 lanes at random rows -- but prefetched a step ahead: a
    // timing-only build with every lane at row t (broadcast, conflict-free) ran lstm_fwd 770 vs 786 us,
    // 0.4% of the step, profiles/r6_bcast; a private table per lane would cost the kernel its occupancy)
    const int o1 = valid ? pos1[rb0] : 0, o2 = valid ? pos2[rb0] : 0;
    const char* tb1 = reinterpret_cast<const char*>(ids_all) + ((q * 2) * R + o1) * 8;
    const char* tb2 = reinterpret_cast<const char*>(ids_all) + ((q * 2 + 1) * R + o2) * 8;
    const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(wrows), (short)0, (int)wbytes,
                                                      0x00020000);
    struct XR {
      uint32_t w;
      uint64_t a, b;
    };
    XR ra, rb;
    auto load_xr = [&](int t, XR& r) __attribute__((always_inline)) {
      // (t is wave-uniform but derived from the wave index: without readfirstlane the soffset operand got a
      // waterfall loop per load)
      r.w = __builtin_amdgcn_raw_buffer_load_b32(rw, wvo, __builtin_amdgcn_readfirstlane(t * 16), 0);
      r.a = *reinterpret_cast<const uint64_t*>(tb1 + t * 8);
      r.b = *reinterpret_cast<const uint64_t*>(tb2 + t * 8);
    };
    auto step_xr = [&](const int tau, const XR& r0) __attribute__((always_inline)) {
      XR r = r0;
      asm volatile("" : "+v"(r.w), "+v"(r.a), "+v"(r.b));
      const uint32_t xw[2] = {(r.w | (uint32_t)r.a | (uint32_t)r.b) & vm,
                              ((uint32_t)(r.a >> 32) | (uint32_t)(r.b >> 32)) & vm};
      step_bf(tau, xw);
    };
    auto xpair = [&](int tau) __attribute__((always_inline)) {
      load_xr(tof(tau + 1), rb);
      __builtin_amdgcn_sched_barrier(0);
      step_xr(tau, ra);
      __builtin_amdgcn_sched_barrier(0);
      load_xr(tof(min(tau + 2, te - 1)), ra);
      __builtin_amdgcn_sched_barrier(0);
      step_xr(tau + 1, rb);
      __builtin_amdgcn_sched_barrier(0);
    };
    load_xr(tof(tb), ra);
    int tau = tb;
    if (te - tb >= 2) {
      xpair(tb);
      tau = tb + 2;
    }
    for (; tau + 1 < te; tau += 2) xpair(tau);
    if (tau < te) step_xr(tau, ra);
    return;
  }
  if constexpr (!FG) {
    u16x4_t ra[NX / 4], rb[NX / 4];
    auto load_raw = [&](int t, u16x4_t* r) {
      const unsigned short* xp = xg + ((uint32_t)(tile * L + t) * 64 + lane) * NX;
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) r[c] = *reinterpret_cast<const u16x4_t*>(xp + 4 * c);
    };
    auto step_raw = [&](const int tau, const u16x4_t* r) __attribute__((always_inline)) {
      // the empty asm pins the conversion here: pure shifts / ands were otherwise hoisted above the
      // sched_barrier into the previous step, with a vmcnt(0) wait for this prefetch in front of them
      u16x4_t rr[NX / 4];
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) {
        rr[c] = r[c];
        asm volatile("" : "+v"(rr[c]));
      }
      uint32_t xw[NX / 2];
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) {
        const uint2 v = __builtin_bit_cast(uint2, rr[c]);
        xw[2 * c] = v.x;
        xw[2 * c + 1] = v.y;
      }
      step_bf(tau, xw);
    };
    // pair structure as below: sched_barrier pins each prefetch ahead of the step it overlaps, and the
    // first pair is peeled so the loop header is entered with the same outstanding-VMEM state from
    // the preheader and the latch (the waitcnt pass can then count precisely)
    auto rpair = [&](int tau) __attribute__((always_inline)) {
      load_raw(tof(tau + 1), rb);
      __builtin_amdgcn_sched_barrier(0);
      step_raw(tau, ra);
      __builtin_amdgcn_sched_barrier(0);
      load_raw(tof(min(tau + 2, te - 1)), ra);
      __builtin_amdgcn_sched_barrier(0);
      step_raw(tau + 1, rb);
      __builtin_amdgcn_sched_barrier(0);
    };
    load_raw(tof(tb), ra);
    int tau = tb;
    if (te - tb >= 2) {
      rpair(tb);
      tau = tb + 2;
    }
    for (; tau + 1 < te; tau += 2) rpair(tau);
    if (tau < te) step_raw(tau, ra);
    return;
  }
  float xa[NX], xb[NX];
  // sched_barrier pins each prefetch ahead of the step it overlaps (the machine scheduler would
  // otherwise sink the loads next to their uses to save registers)
  auto pair = [&](int tau) __attribute__((always_inline)) {
    load_x(tof(tau + 1), xb);
    __builtin_amdgcn_sched_barrier(0);
    step(tau, xa);
    __builtin_amdgcn_sched_barrier(0);
    load_x(tof(min(tau + 2, L - 1)), xa);
    __builtin_amdgcn_sched_barrier(0);
    step(tau + 1, xb);
    __builtin_amdgcn_sched_barrier(0);
  };
  load_x(tof(0), xa);
  int tau = 0;
  // first pair peeled: the loop header is then entered with the same outstanding-VMEM state from
  // the preheader and the latch, so the waitcnt pass can count precisely.
  if (L >= 2) {
    pair(0);
    tau = 2;
  }
  for (; tau + 1 < L; tau += 2) pair(tau);
  if (tau < L) step(tau, xa);
}

// ------------------------------------------------------------------------------------------
// bf16 forward output, lane layout [tile][dir][t][U4][64] -> natural rows [seq][t][2U] (the
// attention input, model/graph.py:49 concat of the two directions).  One workgroup per 16-sequence
// tile: the tile's contiguous input block lands in LDS by LDS-DMA; each sequence's output rows are
// one contiguous run written with coalesced dwords (16 threads per sequence).
// ------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(256) void h_natural_kernel(const unsigned short* __restrict__ rec,
                                                        const unsigned char* __restrict__ dmask, int L,
                                                        float inv_kp, unsigned short* __restrict__ hnat) {
  constexpr int U4 = U / 4, PIECE = U4 * 64 * 2;   // bytes of one (dir, step) h slot
  extern __shared__ __attribute__((aligned(16))) unsigned short lds_h[];   // h [2][L][U4][64], keep bits
  const int tile = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // 1) the h slots of the tile's step records ([2][L][2][U4][64]) and its keep bits [2][L][64] -> LDS
  //    by LDS-DMA (16 B per lane, one piece per wave instruction), all in flight
  const int hbytes = 2 * L * PIECE, hpad = (hbytes + 1023) & ~1023, mbytes = dmask ? 2 * L * 64 : 0;
  const char* src = reinterpret_cast<const char*>(rec) + (size_t)tile * 2 * hbytes;
  char* lds = reinterpret_cast<char*>(lds_h);
  for (int k = wave; k < 2 * L; k += 4)
    if (lane * 16 < PIECE)
      __builtin_amdgcn_global_load_lds(src + (size_t)k * 2 * PIECE + lane * 16, lds + k * PIECE, 16, 0, 0);
  if (dmask) {
    const char* msrc = reinterpret_cast<const char*>(dmask) + (size_t)tile * mbytes;
    for (int k = wave; k * 1024 < mbytes; k += 4) {
      const int off = k * 1024 + lane * 16;
      if (off < mbytes) __builtin_amdgcn_global_load_lds(msrc + off, lds + hpad + k * 1024, 16, 0, 0);
    }
  }
  __syncthreads();
  const unsigned char* keep = reinterpret_cast<const unsigned char*>(lds + hpad);
  // 2) natural rows: thread (sequence n = tid / 16, part) writes dwords part, part + 16, ... of n's
  //    contiguous run [L][2U] (dword = features (2p, 2p + 1) of one step); DropoutWrapper output
  //    keep ? bf16(h / keep_prob) : 0 (model/graph.py:36-38)
  const int n = threadIdx.x >> 4, part = threadIdx.x & 15;
  uint32_t* dst = reinterpret_cast<uint32_t*>(hnat + ((size_t)tile * 16 + n) * L * 2 * U);
  for (int i = part; i < L * U; i += 16) {
    const int t = i / U, f = 2 * (i - t * U);
    uint32_t v = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int fe = f + e, d = fe >= U ? 1 : 0, u = fe - d * U;
      const int li = (u & 3) * 16 + n;
      unsigned short x = lds_h[((d * L + t) * U4 + (u >> 2)) * 64 + li];
      if (dmask) x = ((keep[(d * L + t) * 64 + li] >> (u >> 2)) & 1u) ? f2bf(bf2f(x) * inv_kp) : (unsigned short)0;
      v |= (uint32_t)x << (16 * e);
    }
    dst[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// dW slab layout per (block, dir): D[gc][f], gc in [0, 4U), f in [0, DIN + U + 1) where
// f < DIN are x features, DIN..DIN+U-1 the h units and DIN+U the bias.
// dH layouts (dh_lane): 0 = natural [S][L][2U] (attn_bwd), 1 = the step-record lane layout
// [tiles][2][L][U4][64] (rec_attn_bwd: coalesced 128-B rows per (step, m))
// 2 waves/SIMD where the register set fits in 256 without spilling (the default u=20 / 5-d words
// case); the wider instantiations keep 1 wave and no spills
template <int U, int NX>
struct BwdWaves {
  static constexpr int value = (U <= 20 && NX == 4) ? 2 : 1;
};
// WG: trained word table (word-row gradients by global atomics).  A template flag rather than a
// runtime branch: the join after a skipped atomic block made LLVM drain every outstanding load
// (s_waitcnt vmcnt(0), a register of that block is reused) on every step, prefetch included.
// PM (bf16 only): dH arrives in the step-record lane layout ALREADY multiplied by the DropoutWrapper
// scale (rec_attn_bwd), and the BPTT runs the lean step below (raw bf16 operands, no keep bits, no
// per-lane validity selects, uniform per-step addresses).
// (The attention backward fused into this kernel and per-wave LDS position tables were built and measured
// slower -- profiles/r4_fused_attn, README "negative results"; removed.)
// XD (with PM): direct x -- word features from the word rows, position features from LDS
// tables (see xd_build); no xg record.
template <int U, int NX, bool BF16, bool WG = false, bool PM = false, bool XD = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BwdWaves<U, NX>::value))) void lstm_bwd_kernel(
    const int* __restrict__ inst, int S, const int* __restrict__ word, const int* __restrict__ pos1,
    const int* __restrict__ pos2, int L, const float* __restrict__ wemb, int E,
    const float* __restrict__ p1emb, const float* __restrict__ p2emb, int PD,
    const typename FragT<BF16>::type* __restrict__ apack, const typename FragT<BF16>::type* __restrict__ a2pack,
    const float* __restrict__ bias, const typename FragT<BF16>::elem* __restrict__ hraw,
    const typename CT<BF16>::type* __restrict__ cst, const typename FragT<BF16>::elem* __restrict__ dH,
    float* __restrict__ dw_slab,
    float* __restrict__ dpos_slab, float* __restrict__ dwemb, const unsigned char* __restrict__ dmask, uint32_t seed,
    uint32_t thr, float inv_kp, int drop, unsigned short* __restrict__ dxp, const unsigned short* __restrict__ xg,
    int dh_lane, const int* __restrict__ tlen, const int* __restrict__ slen, int wblank,
    const unsigned short* __restrict__ wrows, uint32_t wbytes) {
  static_assert(!XD || (BF16 && PM && NX == 4), "direct x runs in the lean bf16 BPTT (4 x slots)");
  using Sh = Shape<U, NX, BF16>;
  using frag = typename FragT<BF16>::type;
  using elem = typename FragT<BF16>::elem;
  constexpr int U4 = Sh::U4, KPL = Sh::KPL, NKS = Sh::NKS, NMT = Sh::NMT, NMT2 = Sh::NMT2,
                NKS2 = Sh::NKS2, G4 = Sh::G4, GT = Sh::GT, RS = Sh::RS;
  const int DIN = E + 2 * PD;
  const int NF = DIN + U + 1;            // dW feature columns (incl. bias)
  // WG: the padding row (BLANK, ~1/3 of all tokens) is summed in registers and added once per lane
  // group at the end -- as per-token global atomics every wave hit the same two cache lines (one L2
  // channel): 57 ms per call at 256 episodes instead of ~0.1 ms
  float bacc[NX];
#pragma unroll
  for (int xi = 0; xi < NX; ++xi) bacc[xi] = 0.f;
  const int FT = (NF + 15) / 16;         // dW N-tiles (runtime, <= FTMAX)
  constexpr int FTMAX = (4 * NX + U + 1 + 15) / 16;
  constexpr int NA = NMT * NKS * 64, NA2 = NMT2 * NKS2 * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, n = lane & 15;
  // longest work first (as lstm_fwd): the backward direction's workgroups (all L steps) dispatch first, the forward
  // direction's ragged tile groups in descending length
  const int dir = 1 - (int)blockIdx.y;
  const int ntiles = (S + 15) / 16;
  const int ngroups = (ntiles + 3) / 4;
  const int P2 = 2 * L;  // pos table rows

  // ---- LDS carve: [A packs][bias 4U][xpose 4 waves x XROWS x RS][dpos 2*P2*PD]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  frag* lA = reinterpret_cast<frag*>(smem);
  frag* lA2 = lA + NA;
  float* lbias = reinterpret_cast<float*>(lA2 + NA2);
  size_t off = (size_t)(NA + NA2) * sizeof(frag) + 4 * U * sizeof(float);
  off = (off + 15) & ~(size_t)15;
  constexpr int XROWS = GT * 16 + FTMAX * 16;
  constexpr int NSLP = (U4 + NX + 1) & ~1;               // XH slots per lane: U4 h, NX x (+1 pad)
  constexpr int FTA = BF16 ? (4 * NSLP + 1 + 15) / 16 : FTMAX;
  // +4 elements: row stride != 0 mod 32 banks.  (A bank-model stride for the dG image, 92 at GT 5, halves
  // its modelled transposed-read conflicts but measured neutral, 1420 vs 1413 us.)
  constexpr int GCP = GT * 16 + 4, FCP = FTA * 16 + 4;
  constexpr int WSTRIDE = XROWS * RS;   // per-wave staging region (elements)
  elem* xp_all = reinterpret_cast<elem*>(smem + off);
  elem* dgT = xp_all + (size_t)wave * WSTRIDE;
  elem* xhT = dgT + GT * 16 * RS;
  // bf16 dW staging: a [32 samples][GCP] dG image and a [32 samples][FCP] [x;h;1] image (two steps
  // x 16 sequences), lane-permuted columns so each lane writes its values with a few 8-/4-byte
  // stores (lane (q, n): row 16 (tau & 1) + n, dG columns q*4U4 + 4m + g4, XH columns q*NSLP + slot;
  // the old [gate row][sample] staging took 20 + 9 ds_write_b16 per step).  Both MFMA operands come
  // back through ds_read_b64_tr_b16 (K = the pair's 32 samples, 16x16x32: the 16x16x16 form with
  // K = one step measured 25% slower, half the MFMA rate).
  static_assert(!BF16 || 32 * (GCP + FCP) <= XROWS * RS, "bf16 dW images exceed the staging region");
  unsigned short* dgI = reinterpret_cast<unsigned short*>(dgT);
  unsigned short* xhI = dgI + 32 * GCP;
  const int tcol = 4 * (n & 3);
  {
    // (the region also holds the final reductions)
    size_t xp = (size_t)4 * WSTRIDE * sizeof(elem);
    const size_t red = (size_t)G4 * (4 * NX + U + 1) * sizeof(float);
    off += xp > red ? xp : red;
  }
  off = (off + 15) & ~(size_t)15;
  float* dpos_lds = reinterpret_cast<float*>(smem + off);   // [2 tables][2L][PD]
  // XD: the block's direct-x position tables (lstm_bwd_lds_bytes mirrors this offset)
  char* xdT = reinterpret_cast<char*>(smem) + ((off + 15) & ~(size_t)15);
  if constexpr (XD) xd_copy(xdT, xg, L);   // (xg = x_gather's global copy of the tables)
  // gate packs / biases pre-scaled as in the forward (fragment index i -> lane i & 63, gate i & 3);
  // the transposed pack (d[x;h] = W dG) keeps the true weights
  for (int i = threadIdx.x; i < NA; i += 256) lA[i] = fscale(apack[(size_t)dir * NA + i], gate_scale(i & 3));
  for (int i = threadIdx.x; i < NA2; i += 256) lA2[i] = a2pack[(size_t)dir * NA2 + i];
  // [unit][gate]
  for (int i = threadIdx.x; i < 4 * U; i += 256) lbias[(i % U) * 4 + i / U] = gate_bias(bias[dir * 4 * U + i], i / U);
  if constexpr (!BF16)
    for (int i = threadIdx.x; i < 2 * P2 * PD; i += 256) dpos_lds[i] = 0.f;
  const int NPF = 2 * PD;   // pos features (bf16 mode: exported to dxp, reduced by pos_grad_kernel)
  // zero the wave's transpose buffers once (pad rows / columns stay zero; bias row = 1)
  for (int i = lane; i < WSTRIDE; i += 64) dgT[i] = to_elem(0.f, (elem*)nullptr);
  wave_lds_sync();
  if constexpr (BF16) {
    if (lane < 32) xhI[lane * FCP + 4 * NSLP] = f2bf(1.f);   // bias column
  } else {
    for (int i = lane; i < 32; i += 64) xhT[(DIN + U) * RS + i] = to_elem(1.f, (elem*)nullptr);
  }
  __syncthreads();

  float bm[NMT][4];   // gate biases of the lane's units (registers, not per-step LDS reads)
#pragma unroll
  for (int m = 0; m < NMT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) bm[m][r] = lbias[(4 * m + q) * 4 + r];
  f32x4_t accw[GT][FTA];
#pragma unroll
  for (int a = 0; a < GT; ++a)
#pragma unroll
    for (int b = 0; b < FTA; ++b) accw[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  XSrc xs[NX];
#pragma unroll
  for (int xi = 0; xi < NX; ++xi) xs[xi] = make_xsrc(4 * xi + q, wemb, E, p1emb, p2emb, PD);
  // lane's element offset inside a dxp [NPF + 1][16] step block: its pos feature's row, or the
  // trash row NPF (word / padding features) -- the per-step stores then need no lane-dependent branch
  int pofs[NX];
#pragma unroll
  for (int xi = 0; xi < NX; ++xi)
    pofs[xi] = ((uint32_t)(xs[xi].sel - 1) < 2u ? 4 * xi + q - E : NPF) * 16 + n;

  for (int gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const int g = dir == 0 ? ngroups - 1 - gi : gi;
    const int tile = g * 4 + wave;
    if (tile >= ntiles) continue;  // no block-level barrier inside the group loop
    const int seq = tile * 16 + n;
    const bool valid = seq < S;
    const long seqc = valid ? seq : S - 1;  // clamped row for unconditional loads
    const long rowbase = (long)inst[seqc] * L;
    // dH element (t, m) of the lane = dH[dh_base + t * dh_ts + m * dh_ms] (wave-uniform layout choice)
    const size_t dh_base = dh_lane ? ((size_t)tile * 2 + dir) * L * U4 * 64 + lane
                                   : (size_t)seqc * L * (2 * U) + dir * U + q;
    const int dh_ts = dh_lane ? U4 * 64 : 2 * U, dh_ms = dh_lane ? 64 : 4;
    const typename CT<BF16>::type* cbase = cst + ((size_t)tile * 2 + dir) * L * U4 * 64 + lane;
    const elem* hbase = hraw + ((size_t)tile * 2 + dir) * L * U4 * 64 + lane;
    // bf16: the forward's step records [t][2][U4][64]: h slot, then c slot (fp16 bits)
    const unsigned short* rbase = reinterpret_cast<const unsigned short*>(hraw) + ((size_t)tile * 2 + dir) * L * 2 * U4 * 64 + lane;
    auto ld_hc = [&](int tt, int m, float& hv, float& cv) {
      if constexpr (BF16) {
        hv = bf2f(rbase[((size_t)tt * 2 * U4 + m) * 64]);
        cv = (float)__builtin_bit_cast(_Float16, rbase[((size_t)tt * 2 * U4 + U4 + m) * 64]);
      } else {
        hv = from_elem(hbase[((size_t)tt * U4 + m) * 64]);
        cv = from_c(cbase[((size_t)tt * U4 + m) * 64]);
      }
    };
    auto tof = [&](int tau) { return dir ? (L - 1 - tau) : tau; };  // processing step -> time
    // bf16: x from the x_gather_kernel rows (one coalesced load per 4 features), no token ids
    auto load_xg = [&](int t, float* xv) {
      const unsigned short* xp = xg + ((uint32_t)(tile * L + t) * 64 + lane) * NX;
#pragma unroll
      for (int c = 0; c < NX / 4; ++c) {
        const u16x4_t v = *reinterpret_cast<const u16x4_t*>(xp + 4 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[4 * c + e] = bf2f(v[e]);
      }
    };
    // software pipeline (fp32 mode): ids two steps ahead, everything else one step ahead
    int wid_c = 0, p1_c = 0, p2_c = 0, wid_n = 0, p1_n = 0, p2_n = 0;
    if constexpr (!BF16) {
      const int t0 = tof(L - 1), t1 = tof(L >= 2 ? L - 2 : 0);
      wid_c = word[rowbase + t0]; p1_c = pos1[rowbase + t0]; p2_c = pos2[rowbase + t0];
      wid_n = word[rowbase + t1]; p1_n = pos1[rowbase + t1]; p2_n = pos2[rowbase + t1];
    }
    const unsigned char* mbase = dmask + (size_t)(tile * 2 + dir) * L * 64 + lane;   // fwd keep bits
    float ccur[U4];
    float dh_rec[U4], dc_rec[U4];
#pragma unroll
    for (int m = 0; m < U4; ++m) dh_rec[m] = dc_rec[m] = 0.f;
    if (!(BF16 && PM) && (L & 1)) {
      // odd L: the tile's first dW chunk {L, L-1} is half filled; clear the dG samples of the missing
      // step (they still hold the previous tile's last chunk)
      if constexpr (BF16) {
#pragma unroll
        for (int m = 0; m < U4; ++m)
          *reinterpret_cast<u16x4_t*>(dgI + (16 + n) * GCP + q * (4 * U4) + 4 * m) = u16x4_t{0, 0, 0, 0};
      } else {
#pragma unroll
        for (int m = 0; m < U4; ++m)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) dgT[(g4 * U + 4 * m + q) * RS + n + 16] = to_elem(0.f, (elem*)nullptr);
      }
    }
    // one BPTT step at processing index tau from its converted inputs (ccur, dh_rec, dc_rec, accw
    // carried by reference); wid / p1 / p2: fp32 mode's token ids (unused in bf16 mode)
    auto compute = [&](const int tau, const int wid, const int p1, const int p2, const float* xv, const float* hp,
                       const float* cprev, const float* dhin) __attribute__((always_inline)) {
      // ---- recompute gates
      frag B[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        B[ks] = fzero<BF16>();
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
          const int idx = ks * KPL + j;
          if (idx < U4)
            fset<BF16>(B[ks], j, hp[idx]);
          else if (idx - U4 < NX)
            fset<BF16>(B[ks], j, xv[idx - U4]);
        }
      }
      float dg[U4][4];
#pragma unroll
      for (int m = 0; m < NMT; ++m) {
        f32x4_t acc = {bm[m][0], bm[m][1], bm[m][2], bm[m][3]};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) acc = mma(lA[(m * NKS + ks) * 64 + lane], B[ks], acc);
        const float ig = sigmoid_l2(acc[0]), jg = tanh_l2(acc[1]), fg = sigmoid_l2(acc[2]), og = sigmoid_l2(acc[3]);
        const float tc = tanh_l2(ccur[m] * (2.f * LOG2E_F));
        const float dh = dh_rec[m] + dhin[m];
        const float dc = dc_rec[m] + dh * og * (1.f - tc * tc);
        const float di = dc * jg, dj = dc * ig, df = dc * cprev[m], d_o = dh * tc;
        dc_rec[m] = dc * fg;
        dg[m][0] = di * ig * (1.f - ig);
        dg[m][1] = dj * (1.f - jg * jg);
        dg[m][2] = df * fg * (1.f - fg);
        dg[m][3] = d_o * og * (1.f - og);
      }
      // ---- d[x;h] = W dG
      frag B2[NKS2];
#pragma unroll
      for (int ks = 0; ks < NKS2; ++ks) {
        B2[ks] = fzero<BF16>();
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
          const int idx = ks * KPL + j;
          if (idx < 4 * U4) fset<BF16>(B2[ks], j, dg[idx >> 2][idx & 3]);
        }
      }
      float dslot[NMT2 * 4];
#pragma unroll
      for (int mt = 0; mt < NMT2; ++mt) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS2; ++ks) acc = mma(lA2[(mt * NKS2 + ks) * 64 + lane], B2[ks], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) dslot[mt * 4 + r] = acc[r];
      }
#pragma unroll
      for (int m = 0; m < U4; ++m) dh_rec[m] = dslot[m];
      // x-feature gradients of the pos features.  bf16: plain coalesced stores into dxp (rows of 16
      // sequences per feature); pos_grad_kernel reduces them with one-hot MFMAs -- per-element LDS
      // float atomics here sat on the recurrence's critical path (~20% of this kernel).  fp32: LDS
      // atomics into the block's pos tables.
      if constexpr (BF16) {
        unsigned short* drow = dxp + (((size_t)dir * ntiles + tile) * L + tof(tau)) * (NPF + 1) * 16;
#pragma unroll
        for (int xi = 0; xi < NX; ++xi) drow[pofs[xi]] = f2bf(valid ? dslot[U4 + xi] : 0.f);
        // (the reduction's position ids come from x_gather_kernel's posb)
      } else {
#pragma unroll
        for (int xi = 0; xi < NX; ++xi) {
          const uint32_t i1 = (uint32_t)(p1 * PD + xs[xi].col), i2 = (uint32_t)((P2 + p2) * PD + xs[xi].col);
          if (valid && (uint32_t)(xs[xi].sel - 1) < 2u) atomicAdd(&dpos_lds[lane_sel(xs[xi].mp2, i1, i2)], dslot[U4 + xi]);
        }
      }
      // word table (global atomics, only when trained)
      if constexpr (WG) {
        if (valid) {
          const int wrow = BF16 ? word[rowbase + tof(tau)] : wid;   // bf16: not pipelined (trained words only)
          const bool pad = wrow == wblank;
#pragma unroll
          for (int xi = 0; xi < NX; ++xi) {
            bacc[xi] += pad ? dslot[U4 + xi] : 0.f;
            if (xs[xi].sel == 0 && !pad) atomicAdd(&dwemb[(long)wrow * E + xs[xi].col], dslot[U4 + xi]);
          }
        }
      }
      if constexpr (BF16) {
        // ---- stage dG / [x;h] (image row 16 * (tau & 1) + n; 8-/4-byte stores), and every second
        // step dW += dG^T [x;h;1] over the pair's 32 samples
        const int rr = 16 * (tau & 1) + n;
        unsigned short* gi = dgI + rr * GCP + q * (4 * U4);
#pragma unroll
        for (int m = 0; m < U4; ++m)
          *reinterpret_cast<u16x4_t*>(gi + 4 * m) =
              u16x4_t{f2bf(dg[m][0]), f2bf(dg[m][1]), f2bf(dg[m][2]), f2bf(dg[m][3])};
        float sl[NSLP];
#pragma unroll
        for (int s = 0; s < NSLP; ++s) sl[s] = s < U4 ? hp[s] : (s < U4 + NX ? xv[s - U4] : 0.f);
        uint32_t* xi32 = reinterpret_cast<uint32_t*>(xhI + rr * FCP + q * NSLP);
#pragma unroll
        for (int p = 0; p < NSLP / 2; ++p) xi32[p] = (uint32_t)f2bf(sl[2 * p]) | ((uint32_t)f2bf(sl[2 * p + 1]) << 16);
        if ((tau & 1) == 0) {
          lds_order();
          // 16x16x32 operands: two transposed reads, samples 8q..8q+3 and 8q+4..8q+7
          auto tr8 = [&](const unsigned short* img, int stride, int c0) {
            const s16x4_t lo = tr_read(img + (8 * q + (n >> 2)) * stride + c0 + tcol);
            const s16x4_t hi = tr_read(img + (8 * q + 4 + (n >> 2)) * stride + c0 + tcol);
            return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                           (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
          };
          u16x8_t fbx[FTA];
#pragma unroll
          for (int b = 0; b < FTA; ++b) fbx[b] = tr8(xhI, FCP, 16 * b);
#pragma unroll
          for (int a = 0; a < GT; ++a) {
            const u16x8_t fa = tr8(dgI, GCP, 16 * a);
#pragma unroll
            for (int b = 0; b < FTA; ++b) accw[a][b] = mfma_bf16(fa, fbx[b], accw[a][b]);
          }
          lds_order();   // the next steps' stores come after these reads (in-order LDS)
        }
      } else {
      // ---- stage (dG, XH) for the dW MFMA: sample column = n + 16 * (tau & 1)
      const int scol = n + 16 * (tau & 1);
#pragma unroll
      for (int m = 0; m < U4; ++m)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          dgT[(g4 * U + 4 * m + q) * RS + scol] = to_elem(dg[m][g4], (elem*)nullptr);
#pragma unroll
      for (int m = 0; m < U4; ++m) xhT[(DIN + 4 * m + q) * RS + scol] = to_elem(hp[m], (elem*)nullptr);
#pragma unroll
      for (int xi = 0; xi < NX; ++xi) {
        const int f = 4 * xi + q;
        if (f < DIN) xhT[f * RS + scol] = to_elem(xv[xi], (elem*)nullptr);
      }
      if ((tau & 1) == 0) {
        // chunk {tau+1, tau} complete (columns 16..31 hold tau+1, 0..15 hold tau).  With L odd
        // the first chunk (tau = L-1) is half filled; the other half is zero because every
        // flush clears the lane's dG columns below.
        wave_lds_sync();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
#pragma unroll
          for (int a = 0; a < GT; ++a) {
            const float fa = from_elem(dgT[(a * 16 + n) * RS + 4 * kk + q]);
#pragma unroll
            for (int b = 0; b < FTMAX; ++b) {
              const float fb = from_elem(xhT[(b * 16 + n) * RS + 4 * kk + q]);
              accw[a][b] = mfma_f32(fa, fb, accw[a][b]);
            }
          }
        }
        wave_lds_sync();   // every later chunk rewrites both column halves: no clearing needed
      }
      }
    };
    if constexpr (BF16 && PM) {
      // ---------------- lean bf16 BPTT (premasked lane-layout dH) ----------------
      // Every per-step address is wave-uniform base + a per-lane constant (saddr loads / stores, no
      // 64-bit VALU address math); h / x stay raw bf16 bits from the load to the B operand and the dW
      // image (v_perm pairs, no f32 round trip); dH needs one shift (it carries the dropout scale).
      const int tu = __builtin_amdgcn_readfirstlane(tile);
      // buffer descriptors over this (tile, dir)'s regions: per-step offsets go in SGPR soffset, the lane's
      // part in a loop-invariant voffset (no per-step VALU address math)
      auto rsrc = [](const void* base, uint32_t bytes) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
      };
      const uint32_t RSTEPB = 2 * U4 * 64 * 2, DSTEPB = U4 * 64 * 2, XSTEPB = 64 * NX * 2, PSTEPB = (NPF + 1) * 16 * 2;
      const auto rrec = rsrc(reinterpret_cast<const unsigned short*>(hraw) + ((size_t)tu * 2 + dir) * L * 2 * U4 * 64,
                             (uint32_t)L * RSTEPB);
      // ragged tiles: the tile's steps [0, Lt) carry attention gradient; the descriptor's range ends there,
      // so dH loads past it return 0 (the backward direction's padding steps in parity mode)
      const int Lt = tlen ? tlen[tu] : L;
      const auto rdh = rsrc(reinterpret_cast<const unsigned short*>(dH) + ((size_t)tu * 2 + dir) * L * U4 * 64,
                            (uint32_t)Lt * DSTEPB);
      const bool lane_reset = slen != nullptr && dir == 1;   // sequence_length semantics (backward direction)
      const int mylen = slen != nullptr ? (valid ? slen[seq] : 0) : L;
      const auto rx = rsrc(XD ? (const unsigned short*)wrows : xg + (size_t)tu * L * 64 * NX,
                           XD ? wbytes : (uint32_t)L * XSTEPB);
      // XD: the lane's word-row dword (padding rows: past the range -> 0) and position-table entries
      const uint32_t wvo = valid ? (uint32_t)rowbase * 16u + 4u * (uint32_t)q : 0x80000000u;
      const char* xtb1 = xdT + ((q * 2) * 2 * L + (valid ? pos1[rowbase] : 0)) * 8;
      const char* xtb2 = xdT + ((q * 2 + 1) * 2 * L + (valid ? pos2[rowbase] : 0)) * 8;
      const uint32_t xvm = valid ? 0xFFFFFFFFu : 0u;   // padding sequences: x = 0
      const auto rdx = rsrc(dxp + ((size_t)dir * ntiles + tu) * L * (NPF + 1) * 16, (uint32_t)L * PSTEPB);
      const int vl2 = lane * 2, vx = lane * NX * 2;
      constexpr int NXW = NX / 2;   // x words (2 features each) per lane and step
      struct Raw {
        uint32_t h[U4], c[U4], d[U4];   // 16-bit loads (upper halves never read)
        uint32_t x[NXW];
        uint64_t pa, pb;                // XD: position-table entries (x[0] = the word dword until bstep)
      };
      auto rload = [&](int tau, Raw& o) __attribute__((always_inline)) {
        const int tn = tof(tau), tp = tof(tau >= 1 ? tau - 1 : 0);
        const int sr = tp * RSTEPB, sd = tn * DSTEPB, sx = tn * XSTEPB;
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          o.h[m] = __builtin_amdgcn_raw_buffer_load_b16(rrec, vl2 + m * 128, sr, 0);
          o.c[m] = __builtin_amdgcn_raw_buffer_load_b16(rrec, vl2 + (U4 + m) * 128, sr, 0);
          o.d[m] = __builtin_amdgcn_raw_buffer_load_b16(rdh, vl2 + m * 128, sd, 0);
        }
        if constexpr (XD) {
          o.x[0] = __builtin_amdgcn_raw_buffer_load_b32(rx, wvo, tn * 16, 0);
          o.pa = *reinterpret_cast<const uint64_t*>(xtb1 + tn * 8);
          o.pb = *reinterpret_cast<const uint64_t*>(xtb2 + tn * 8);
        } else {
#pragma unroll
          for (int k = 0; k < NXW / 2; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rx, vx + 8 * k, sx, 0);
            o.x[2 * k] = (uint32_t)v[0];
            o.x[2 * k + 1] = (uint32_t)v[1];
          }
        }
      };
      auto pkf = [](float a, float b) {   // two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32)
        typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
        const bf2_t v = {(__bf16)a, (__bf16)b};
        return __builtin_bit_cast(uint32_t, v);
      };
      float hcv[U4];   // h_t (bf16 record) of the step being processed: tanh(c_t) = h_t / o_t
      // HASP: the step has a predecessor state (else it is zero: the direction's first step in time, or the
      // SKIP backward direction's tile start).  HI: the step stages into image rows 16..31 and completes
      // the pair (rows 0..15 = the previous step), FLUSH: the pair goes into dW after staging.
      auto bstep = [&](auto hasp_c, auto hi_c, auto flush_c, const int tau, const Raw& X0) __attribute__((always_inline)) {
        constexpr bool HASP = decltype(hasp_c)::value, ODD = decltype(hi_c)::value, FLUSH = decltype(flush_c)::value;
        Raw X = X0;
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          asm volatile("" : "+v"(X.h[m]), "+v"(X.c[m]), "+v"(X.d[m]));
        }
        if constexpr (XD) {   // word dword | the two table entries (disjoint nonzero slots)
          asm volatile("" : "+v"(X.x[0]), "+v"(X.pa), "+v"(X.pb));
          X.x[0] = (X.x[0] | (uint32_t)X.pa | (uint32_t)X.pb) & xvm;
          X.x[1] = ((uint32_t)(X.pa >> 32) | (uint32_t)(X.pb >> 32)) & xvm;
        } else {
#pragma unroll
          for (int k = 0; k < NXW; ++k) asm volatile("" : "+v"(X.x[k]));
        }
        const int t = tof(tau);
        // slot words [h (U4) ; x (NX slots) ; 0]: the gate B operand and the dW image row.  Slot s is the
        // 16-bit half `off` (byte 0 or 2, -1 = zero) of register word `wd`; a pair word is ONE v_perm.
        struct Half {
          uint32_t wd;
          int off;
        };
        auto slot = [&](int sidx) -> Half {
          if (sidx < U4) return HASP ? Half{X.h[sidx], 0} : Half{0u, -1};
          const int xi = sidx - U4;
          if (xi < NX) return Half{X.x[xi >> 1], 2 * (xi & 1)};
          return Half{0u, -1};
        };
        constexpr int NW = NKS * 4;   // B operand words (8 slots per K-step)
        uint32_t bw[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const int s0 = 2 * w, s1 = 2 * w + 1;
          const Half lo = slot(s0), hi = slot(s1);
          if (lo.off < 0 && hi.off < 0) {
            bw[w] = 0u;
          } else if (s0 >= U4 && ((s0 - U4) & 1) == 0 && s1 < U4 + NX) {
            bw[w] = lo.wd;   // an aligned x pair is one loaded word
          } else {           // v_perm: bytes 0-3 of src1 (lo word), 4-7 of src0 (hi word), 0x0C = zero byte
            const uint32_t sl = lo.off < 0 ? 0x0C0Cu : (uint32_t)(lo.off | ((lo.off + 1) << 8));
            const uint32_t sh = hi.off < 0 ? 0x0C0Cu : (uint32_t)((4 + hi.off) | ((5 + hi.off) << 8));
            bw[w] = __builtin_amdgcn_perm(hi.off < 0 ? 0u : hi.wd, lo.off < 0 ? 0u : lo.wd, sl | (sh << 16));
          }
        }
        float cprev[U4], dhin[U4];
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          cprev[m] = HASP ? (float)__builtin_bit_cast(_Float16, (unsigned short)X.c[m]) : 0.f;
          dhin[m] = __builtin_bit_cast(float, X.d[m] << 16);
        }
        // ---- recompute gates
        float dg[U4][4];
#pragma unroll
        for (int m = 0; m < NMT; ++m) {
          f32x4_t acc = {bm[m][0], bm[m][1], bm[m][2], bm[m][3]};
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks)
            acc = mma(lA[(m * NKS + ks) * 64 + lane],
                      __builtin_bit_cast(u16x8_t, u32x4_t{bw[4 * ks], bw[4 * ks + 1], bw[4 * ks + 2], bw[4 * ks + 3]}), acc);
          const float ig = sigmoid_l2(acc[0]), jg = tanh_l2(acc[1]), fg = sigmoid_l2(acc[2]);
          // lean BPTT: tanh(c_t) = h_t / o_t = h_t (1 + 2^-z_o) from the step record's h_t and the o gate's exp
          // (no exp / rcp pair per unit and step for tanh(c_t); h_t is the forward's bf16 h, relative error
          // <= 2^-9).  o = 1 / (1 + e), e = 2^-z_o (z clamped: e stays finite, and where o ~ 0 every use of tc is
          // scaled by o)
          // (the clamp on exp2's result, 2^126: the exp reads the accumulator as the forward's gate exps do, and the
          // v_min needs no canonicalize (fminf(-acc[3], 126) cost a v_max + v_min).  __builtin_amdgcn_fmed3f(-acc[3],
          // -3e38, 126), one v_med3 on the accumulator, failed test_encoder_backward at u = 32: profiles/r6_med3)
          const float eo = fminf(__builtin_amdgcn_exp2f(-acc[3]), 0x1p126f);
          const float og = fast_rcp(1.f + eo);
          const float tc = hcv[m] * (1.f + eo);
          const float dh = dh_rec[m] + dhin[m];
          // (shared products: the step is VALU-issue bound -- README "ISA budget"; 14 instead of 16 ops per unit)
          const float dho = dh * og;
          const float dc = fmaf(dho, fmaf(-tc, tc, 1.f), dc_rec[m]);
          dc_rec[m] = dc * fg;
          const float dci = dc * ig;
          dg[m][0] = dci * fmaf(-jg, ig, jg);          // dc jg ig (1 - ig)
          dg[m][1] = dci * fmaf(-jg, jg, 1.f);         // dc ig (1 - jg^2)
          dg[m][2] = dc * cprev[m] * fmaf(-fg, fg, fg);
          const float dot = dho * tc;
          dg[m][3] = fmaf(-dot, og, dot);              // dh tc og (1 - og)
          ccur[m] = cprev[m];
          hcv[m] = HASP ? bf2f((unsigned short)X.h[m]) : 0.f;   // h_t of the next processed step (time tp)
        }
        uint32_t dgw[2 * U4];   // packed bf16 dG pairs: the W dG operand and the dW image row
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          dgw[2 * m] = pkf(dg[m][0], dg[m][1]);
          dgw[2 * m + 1] = pkf(dg[m][2], dg[m][3]);
        }
        // ---- d[x;h] = W dG
        float dslot[NMT2 * 4];
#pragma unroll
        for (int mt = 0; mt < NMT2; ++mt) {
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < NKS2; ++ks) {
            uint32_t w4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) w4[j] = 4 * ks + j < 2 * U4 ? dgw[4 * ks + j] : 0u;
            acc = mma(lA2[(mt * NKS2 + ks) * 64 + lane], __builtin_bit_cast(u16x8_t, u32x4_t{w4[0], w4[1], w4[2], w4[3]}),
                      acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) dslot[mt * 4 + r] = acc[r];
        }
#pragma unroll
        for (int m = 0; m < U4; ++m) dh_rec[m] = dslot[m];
        if (lane_reset) {   // the row's state before this step (in time order: t + 1) was reset to zero
          const float k = t + 1 < mylen ? 1.f : 0.f;
#pragma unroll
          for (int m = 0; m < U4; ++m) {
            dh_rec[m] *= k;
            dc_rec[m] *= k;
          }
        }
        {   // pos-feature gradients -> dxp rows (word / padding features: the trash row)
          const int sp = t * PSTEPB;
#pragma unroll
          for (int xi = 0; xi < NX; xi += 2) {
            const uint32_t w = pkf(dslot[U4 + xi], xi + 1 < NX ? dslot[U4 + xi + 1] : 0.f);
            __builtin_amdgcn_raw_buffer_store_b16((unsigned short)w, rdx, 2 * pofs[xi], sp, 0);
            if (xi + 1 < NX) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(w >> 16), rdx, 2 * pofs[xi + 1], sp, 0);
          }
        }
        if constexpr (WG) {   // trained word table: global atomics
          if (valid) {
            const int wrow = word[rowbase + t];
            const bool pad = wrow == wblank;
#pragma unroll
            for (int xi = 0; xi < NX; ++xi) {
              bacc[xi] += pad ? dslot[U4 + xi] : 0.f;
              if (xs[xi].sel == 0 && !pad) atomicAdd(&dwemb[(long)wrow * E + xs[xi].col], dslot[U4 + xi]);
            }
          }
        }
        // ---- stage dG / [h;x] into the pair's image rows, flush on the even step
        constexpr int RR = ODD ? 16 : 0;
        uint32_t* gi = reinterpret_cast<uint32_t*>(dgI + (RR + n) * GCP + q * (4 * U4));
#pragma unroll
        for (int w = 0; w < 2 * U4; ++w) gi[w] = dgw[w];
        uint32_t* xi32 = reinterpret_cast<uint32_t*>(xhI + (RR + n) * FCP + q * NSLP);
#pragma unroll
        for (int w = 0; w < NSLP / 2; ++w) xi32[w] = w < NW ? bw[w] : 0u;
        if constexpr (FLUSH) {
          lds_order();
          auto tr8 = [&](const unsigned short* img, int stride, int c0) {
            const s16x4_t lo = tr_read(img + (8 * q + (n >> 2)) * stride + c0 + tcol);
            const s16x4_t hi = tr_read(img + (8 * q + 4 + (n >> 2)) * stride + c0 + tcol);
            return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                           (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
          };
          u16x8_t fbx[FTA];
#pragma unroll
          for (int b = 0; b < FTA; ++b) fbx[b] = tr8(xhI, FCP, 16 * b);
#pragma unroll
          for (int a = 0; a < GT; ++a) {
            const u16x8_t fa = tr8(dgI, GCP, 16 * a);
#pragma unroll
            for (int b = 0; b < FTA; ++b) accw[a][b] = mfma_bf16(fa, fbx[b], accw[a][b]);
          }
          lds_order();
        }
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      // processing steps tau_start .. tau_end (descending; tof maps to time).  Forward direction: from the
      // tile's last valid step (its later steps have zero gradient).  Backward direction: all L (parity) or
      // time [0, Lt) (SKIP).  The last processed step never has a predecessor state.
      const int tau_start = dir == 0 ? Lt - 1 : L - 1;
      const int tau_end = (dir == 1 && slen != nullptr) ? L - Lt : 0;
      const int nst = tau_start - tau_end + 1;
      // dxp rows of the steps not processed: zero (the pos-gradient reduction reads every step)
      for (int t = Lt; t < L; ++t) {
        if (dir == 1 && slen == nullptr) break;
#pragma unroll
        for (int xi = 0; xi < NX; ++xi)
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)0, rdx, 2 * pofs[xi], t * PSTEPB, 0);
      }
#pragma unroll
      for (int m = 0; m < U4; ++m) {   // c and h of the first processed step
        ccur[m] = (float)__builtin_bit_cast(
            _Float16, (unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rrec, vl2 + (U4 + m) * 128, tof(tau_start) * RSTEPB, 0));
        hcv[m] = bf2f((unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rrec, vl2 + m * 128, tof(tau_start) * RSTEPB, 0));
      }
      Raw A, B;
      rload(tau_start, A);
      int k = 0;   // processed steps so far: pairs (k, k + 1) -> image rows 0..15 / 16..31
      for (; k + 2 < nst; k += 2) {
        rload(tau_start - k - 1, B);
        __builtin_amdgcn_sched_barrier(0);
        bstep(T_{}, F_{}, F_{}, tau_start - k, A);
        __builtin_amdgcn_sched_barrier(0);
        rload(tau_start - k - 2, A);
        __builtin_amdgcn_sched_barrier(0);
        bstep(T_{}, T_{}, T_{}, tau_start - k - 1, B);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (nst - k == 2) {
        rload(tau_end, B);
        __builtin_amdgcn_sched_barrier(0);
        bstep(T_{}, F_{}, F_{}, tau_start - k, A);
        __builtin_amdgcn_sched_barrier(0);
        bstep(F_{}, T_{}, T_{}, tau_end, B);
      } else {   // a lone last step: its pair's other half (rows 16..31) holds flushed data -> zero dG
#pragma unroll
        for (int m = 0; m < U4; ++m)
          *reinterpret_cast<u16x4_t*>(dgI + (16 + n) * GCP + q * (4 * U4) + 4 * m) = u16x4_t{0, 0, 0, 0};
        bstep(F_{}, F_{}, T_{}, tau_end, A);
      }
    } else if constexpr (!BF16) {
    float xv[NX], hp[U4], cprev[U4], dhin[U4];
    {
      const int t = tof(L - 1), tp = tof(L >= 2 ? L - 2 : 0);
      const uint32_t bits = drop ? (uint32_t)mbase[(size_t)t * 64] : 0xFFu;
      if constexpr (BF16) {
        load_xg(t, xv);
      } else {
#pragma unroll
        for (int xi = 0; xi < NX; ++xi) xv[xi] = gather_x(xs[xi], xrow(wid_c, p1_c, p2_c, E, PD));
      }
#pragma unroll
      for (int m = 0; m < U4; ++m) {
        float hdummy, cp, hv;
        ld_hc(t, m, hdummy, ccur[m]);
        ld_hc(tp, m, hv, cp);
        cprev[m] = L >= 2 ? cp : 0.f;
        hp[m] = (L >= 2 && valid) ? hv : 0.f;
        const float dv = from_elem(dH[dh_base + (size_t)t * dh_ts + m * dh_ms]);
        const bool keep = (bits >> m) & 1u;
        dhin[m] = (valid && keep) ? dv * inv_kp : 0.f;
      }
    }
    for (int tau = L - 1; tau >= 0; --tau) {
      // ---- prefetch step tau-1 (x, h_{tau-2}, c_{tau-2}, dH_{tau-1}) and ids of tau-2
      const int taun = tau >= 1 ? tau - 1 : 0;
      const int taunn = tau >= 2 ? tau - 2 : 0;
      const bool n_has_prev = tau >= 2;
      const int tn = tof(taun), tnp = tof(taunn), tnn = tof(taunn);
      int wid_nn = 0, p1_nn = 0, p2_nn = 0;
      if constexpr (!BF16) {
        wid_nn = word[rowbase + tnn];
        p1_nn = pos1[rowbase + tnn];
        p2_nn = pos2[rowbase + tnn];
      }
      float xv_n[NX], hp_n[U4], cprev_n[U4], dhin_n[U4];
      const uint32_t bits_n = drop ? (uint32_t)mbase[(size_t)tn * 64] : 0xFFu;
      if constexpr (BF16) {
        load_xg(tn, xv_n);
      } else {
#pragma unroll
        for (int xi = 0; xi < NX; ++xi) xv_n[xi] = gather_x(xs[xi], xrow(wid_n, p1_n, p2_n, E, PD));
      }
#pragma unroll
      for (int m = 0; m < U4; ++m) {
        float hv, cp;
        ld_hc(tnp, m, hv, cp);
        cprev_n[m] = n_has_prev ? cp : 0.f;
        hp_n[m] = (n_has_prev && valid) ? hv : 0.f;
        const float dv = from_elem(dH[dh_base + (size_t)tn * dh_ts + m * dh_ms]);
        const bool keep = (bits_n >> m) & 1u;
        dhin_n[m] = (valid && keep) ? dv * inv_kp : 0.f;
      }
      compute(tau, wid_c, p1_c, p2_c, xv, hp, cprev, dhin);
      // ---- rotate the pipeline
#pragma unroll
      for (int m = 0; m < U4; ++m) {
        ccur[m] = cprev[m];
        cprev[m] = cprev_n[m];
        hp[m] = hp_n[m];
        dhin[m] = dhin_n[m];
      }
#pragma unroll
      for (int xi = 0; xi < NX; ++xi) xv[xi] = xv_n[xi];
      wid_c = wid_n; p1_c = p1_n; p2_c = p2_n;
      wid_n = wid_nn; p1_n = p1_nn; p2_n = p2_nn;
    }
    } else {
      // bf16: ping-pong RAW step buffers (2x unrolled).  The prefetch of step tau-1 lands in the other
      // buffer and is converted only when that step runs; the empty asm on the raw registers pins the
      // conversion there (pure conversions were otherwise hoisted into the previous step together
      // with a wait for the prefetch, i.e. no overlap).
      struct RawB {
        unsigned short h[U4], c[U4], d[U4];   // h / c of processing step tau-1, dH of step tau
        unsigned short kb;                     // keep bits of step tau (| kor in bstep, after the pin)
        u16x4_t x[NX / 4];                     // x_gather row of step tau
      };
      const unsigned char* kbase = drop ? mbase : reinterpret_cast<const unsigned char*>(rbase);
      const uint32_t kor = drop ? 0u : 0xFFu;
      auto rload = [&](int tau, RawB& o) __attribute__((always_inline)) {
        const int tn = tof(tau), tp = tof(tau >= 1 ? tau - 1 : 0);
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          o.h[m] = rbase[((size_t)tp * 2 * U4 + m) * 64];
          o.c[m] = rbase[((size_t)tp * 2 * U4 + U4 + m) * 64];
          o.d[m] = reinterpret_cast<const unsigned short*>(dH)[dh_base + (size_t)tn * dh_ts + m * dh_ms];
        }
        o.kb = kbase[(size_t)tn * 64];
        const unsigned short* xp = xg + ((uint32_t)(tile * L + tn) * 64 + lane) * NX;
#pragma unroll
        for (int c = 0; c < NX / 4; ++c) o.x[c] = *reinterpret_cast<const u16x4_t*>(xp + 4 * c);
      };
      auto bstep = [&](int tau, const RawB& X0) __attribute__((always_inline)) {
        RawB X = X0;
#pragma unroll
        for (int m = 0; m < U4; ++m) asm volatile("" : "+v"(X.h[m]), "+v"(X.c[m]), "+v"(X.d[m]));
        asm volatile("" : "+v"(X.kb));
#pragma unroll
        for (int c = 0; c < NX / 4; ++c) asm volatile("" : "+v"(X.x[c]));
        const bool hasp = tau >= 1;
        float xv[NX], hp[U4], cprev[U4], dhin[U4];
#pragma unroll
        for (int c = 0; c < NX / 4; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) xv[4 * c + e] = bf2f(X.x[c][e]);
#pragma unroll
        for (int m = 0; m < U4; ++m) {
          hp[m] = (hasp && valid) ? bf2f(X.h[m]) : 0.f;
          cprev[m] = hasp ? (float)__builtin_bit_cast(_Float16, X.c[m]) : 0.f;
          dhin[m] = (valid && ((((uint32_t)X.kb | kor) >> m) & 1u)) ? bf2f(X.d[m]) * inv_kp : 0.f;
        }
        compute(tau, 0, 0, 0, xv, hp, cprev, dhin);
#pragma unroll
        for (int m = 0; m < U4; ++m) ccur[m] = cprev[m];
      };
#pragma unroll
      for (int m = 0; m < U4; ++m)   // c of the first processed step
        ccur[m] = (float)__builtin_bit_cast(_Float16, rbase[((size_t)tof(L - 1) * 2 * U4 + U4 + m) * 64]);
      RawB A, B;
      rload(L - 1, A);
      int tau = L - 1;
      for (; tau >= 1; tau -= 2) {
        rload(tau - 1, B);
        __builtin_amdgcn_sched_barrier(0);
        bstep(tau, A);
        __builtin_amdgcn_sched_barrier(0);
        rload(tau >= 2 ? tau - 2 : 0, A);
        __builtin_amdgcn_sched_barrier(0);
        bstep(tau - 1, B);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (tau == 0) bstep(0, A);
    }
  }
  if constexpr (WG) {   // the padding row: sum over the lane group's 16 sequences, one atomic per feature
#pragma unroll
    for (int xi = 0; xi < NX; ++xi) {
      const float v = group16_sum(bacc[xi]);
      if (n == 0 && xs[xi].sel == 0 && wblank >= 0) atomicAdd(&dwemb[(long)wblank * E + xs[xi].col], v);
    }
  }
  // ---- reduce dW across the 4 waves through LDS (reuse the transpose region as f32)
  __syncthreads();
  float* red = reinterpret_cast<float*>(xp_all);
  const int REDN = G4 * NF;
  for (int i = threadIdx.x; i < REDN; i += 256) red[i] = 0.f;
  __syncthreads();
  // bf16: un-permute the image columns (dG column c -> gate row, XH column -> feature; -1 = pad)
  int fmap[FTA];
#pragma unroll
  for (int b = 0; b < FTA; ++b) {
    const int c = b * 16 + n;
    if constexpr (BF16) {
      const int qq = c / NSLP, s = c - qq * NSLP;
      fmap[b] = c == 4 * NSLP ? DIN + U
                : c > 4 * NSLP ? -1
                : s < U4       ? DIN + 4 * s + qq
                : (s < U4 + NX && 4 * (s - U4) + qq < DIN) ? 4 * (s - U4) + qq
                               : -1;
    } else {
      fmap[b] = (b < FT && c < NF) ? c : -1;
    }
  }
  ordered_wave_accumulate(wave, 4, [&] {   // deterministic summation order
#pragma unroll
    for (int a = 0; a < GT; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = a * 16 + 4 * q + r;
        int gc = c;
        if constexpr (BF16) {
          const int qq = c / (4 * U4), rem = c - qq * (4 * U4);
          gc = (rem & 3) * U + 4 * (rem >> 2) + qq;
        }
        if (c >= G4) continue;
#pragma unroll
        for (int b = 0; b < FTA; ++b)
          if (fmap[b] >= 0) red[gc * NF + fmap[b]] += accw[a][b][r];
      }
  });
  float* slab = dw_slab + ((size_t)blockIdx.x * 2 + dir) * REDN;
  for (int i = threadIdx.x; i < REDN; i += 256) slab[i] = red[i];
  if constexpr (!BF16) {
    float* ps = dpos_slab + ((size_t)blockIdx.x * 2 + dir) * 2 * P2 * PD;
    for (int i = threadIdx.x; i < 2 * P2 * PD; i += 256) ps[i] = dpos_lds[i];
  }
}

// ------------------------------------------------------------------------------------------
// pos-table gradients (bf16 mode): dpos_tb[p][c] = sum over (s, t) with pos_tb[s][t] == p of
// dx[s][t][c], both directions.  As a GEMM: D[p][c] += OneHot[p][sample] * DX[sample][c] with
// K = 32 samples (2 steps x 16 sequences of a tile) per v_mfma_f32_16x16x32_bf16; the one-hot A
// fragments are built in registers from the position ids lstm_bwd stored next to dx (shared by
// the two directions and, per position tile, by both tables' columns).  NPT = position tiles
// (2L <= 16 * NPT, ids < 256).
// ------------------------------------------------------------------------------------------
template <int NPT>
__global__ __launch_bounds__(256) void pos_grad_kernel(const unsigned short* __restrict__ dxp,
                                                       const unsigned short* __restrict__ posb, int S, int L, int PD,
                                                       float* __restrict__ slab) {
  __shared__ float red[4][2 * 16 * NPT * 8];   // per-wave partials (summed in fixed order: deterministic)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i16 = lane & 15, kg = lane >> 4;
  const int ntiles = (S + 15) / 16, npairs = (L + 1) / 2, NPF = 2 * PD, P2 = 2 * L;
  const long items = (long)ntiles * npairs;
  const size_t dstride = (size_t)ntiles * L * (NPF + 1) * 16;   // one direction of dxp (+ trash row)
  const int half = (kg & 1) * 8, sstep = kg >> 1;         // fragment k = 8 kg + e <-> (step, seq)
  const int col = i16 < NPF ? i16 : NPF - 1;
  f32x4_t acc[2][NPT];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) acc[tb][pt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const long stride = (long)gridDim.x * 4;
  long it = (long)blockIdx.x * 4 + wave;
  // three independent 16-byte loads per item (dx of both directions, position ids); software
  // pipelined one item ahead
  auto load = [&](long item, u16x8_t& b0, u16x8_t& b1, u16x8_t& pp, bool& zero) {
    const long itc = item < items ? item : items - 1;
    const int tile = (int)(itc / npairs), pr = (int)(itc - (long)tile * npairs);
    const int t = 2 * pr + sstep;
    const int tc = t < L ? t : L - 1;
    const size_t o = (((size_t)tile * L + tc) * (NPF + 1) + col) * 16 + half;
    b0 = *reinterpret_cast<const u16x8_t*>(dxp + o);
    b1 = *reinterpret_cast<const u16x8_t*>(dxp + dstride + o);
    pp = *reinterpret_cast<const u16x8_t*>(posb + ((size_t)tile * L + tc) * 16 + half);
    zero = t >= L || i16 >= NPF;
  };
  u16x8_t nb0, nb1, npp;
  bool nz;
  load(it, nb0, nb1, npp, nz);
  for (; it < items; it += stride) {
    u16x8_t b0 = nb0, b1 = nb1, pp = npp;
    const bool z = nz;
    load(it + stride, nb0, nb1, npp, nz);
    if (z) b0 = b1 = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    // one-hot A rows: element e of the lane's row p = pt*16 + i16 is 1 iff pos(e) == p.  Pair bits
    // m = (1 << tile(e0)) | (1 << (16 + tile(e1))) for samples landing on row i16 (bit 15 / 31 =
    // no hit, never a tile index); a tile's packed bf16 pair is then ((m >> pt) & 0x10001) * 0x3F80.
    uint32_t m1[4], m2[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t v0 = pp[2 * w], v1 = pp[2 * w + 1];
      const uint32_t a0 = v0 & 0xFF, a1 = v1 & 0xFF, c0 = v0 >> 8, c1 = v1 >> 8;
      const uint32_t ha0 = (a0 & 15) == (uint32_t)i16 ? (a0 >> 4) : 15u;
      const uint32_t ha1 = (a1 & 15) == (uint32_t)i16 ? (a1 >> 4) : 15u;
      const uint32_t hc0 = (c0 & 15) == (uint32_t)i16 ? (c0 >> 4) : 15u;
      const uint32_t hc1 = (c1 & 15) == (uint32_t)i16 ? (c1 >> 4) : 15u;
      m1[w] = (1u << ha0) | (1u << (16 + ha1));
      m2[w] = (1u << hc0) | (1u << (16 + hc1));
    }
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      uint32_t w1[4], w2[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        w1[w] = __umul24((m1[w] >> pt) & 0x10001u, 0x3F80u);
        w2[w] = __umul24((m2[w] >> pt) & 0x10001u, 0x3F80u);
      }
      u16x8_t a1, a2;
      __builtin_memcpy(&a1, w1, 16);
      __builtin_memcpy(&a2, w2, 16);
      acc[0][pt] = mfma_bf16(a1, b0, acc[0][pt]);
      acc[0][pt] = mfma_bf16(a1, b1, acc[0][pt]);
      acc[1][pt] = mfma_bf16(a2, b0, acc[1][pt]);
      acc[1][pt] = mfma_bf16(a2, b1, acc[1][pt]);
    }
  }
  // D[row = 4 kg + r][col = i16] of tile pt = (position pt*16 + row, feature column i16); table tb
  // owns columns [tb*PD, tb*PD + PD)
  // (every (table, p, c) is owned by exactly one lane of the wave)
#pragma unroll
  for (int tb = 0; tb < 2; ++tb) {
    const int c = i16 - tb * PD;
    if (c >= 0 && c < PD) {
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = pt * 16 + 4 * kg + r;
          if (p < P2) red[wave][(tb * P2 + p) * PD + c] = acc[tb][pt][r];
        }
    }
  }
  __syncthreads();
  float* out = slab + (size_t)blockIdx.x * 2 * P2 * PD;
  for (int i = threadIdx.x; i < 2 * P2 * PD; i += 256) out[i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// ------------------------------------------------------------------------------------------
// pos-table gradients, shifted-position form (bf16 mode).  FewRel position ids are a shifted arange
// per sequence: pos[s][t] = o_s + t (o_s = L - entity index, model/base.py / util/data_loader.py:
// pos = j - p + L), checked on the host (ops/sampler.py::DeviceDataset.pos_shift).  Then
//   dpos[p][c] = sum_t G[p - t][t][c],   G[o][t][c] = sum_{s : o_s = o} dx[s][t][c]
// and G is a GEMM with K = sequences and a per-SEQUENCE one-hot: one v_mfma_f32_16x16x32_bf16 covers
// 32 sequences x 16 (t, c) columns, instead of 32 (sequence, step) samples x 16 positions in the
// general kernel above -- ~37x fewer MFMAs and one-hot builds.  o_s <= L, so NRT = ceil((L+1)/16)
// row tiles.  Stage 1 (this kernel): wave = (table, 16-column tile, chunk of K-steps), partial G per
// chunk -> gpart[chunk][table][NRT*16][NT*16].  Stage 2 (pos_shift_finish): one workgroup per output
// (table, p, c) sums chunks and the diagonal in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------
template <int NRT>
__global__ __launch_bounds__(256) void pos_shift_gemm_kernel(const unsigned short* __restrict__ dxp,
                                                             const unsigned short* __restrict__ posb, int S, int L,
                                                             int PD, int kps, float* __restrict__ gpart,
                                                             const int* __restrict__ tlen) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, n = lane & 15;
  const int ntiles = (S + 15) / 16, NPF = 2 * PD;
  const int ncol = L * PD, NT = (ncol + 15) / 16;
  const int gw = blockIdx.x * 4 + wave;   // (table, column tile)
  if (gw >= 2 * NT) return;               // no workgroup barrier in this kernel
  const int tb = gw / NT, nt = gw - tb * NT;
  const int ci = nt * 16 + n;             // this lane's B column = (step t, feature c)
  const bool cval = ci < ncol;
  const int t = cval ? ci / PD : 0;
  const int f = tb * PD + (cval ? ci - t * PD : 0);
  const size_t dstride = (size_t)ntiles * L * (NPF + 1) * 16;   // dxp rows: NPF features + trash row
  const int half = (q & 1) * 8, sh = tb * 8;
  const int ksteps = (ntiles + 1) / 2;   // 32 sequences (2 tiles) per K-step
  const int k0 = blockIdx.y * kps, k1 = min(ksteps, k0 + kps);
  f32x4_t acc[NRT];
#pragma unroll
  for (int pt = 0; pt < NRT; ++pt) acc[pt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // B fragment: lane (q, n) holds sequences 8(q&1)..+7 of tile 2ks + (q>>1) at column n (16 B, both
  // directions); the one-hot A row n of tile pt marks the sequences whose offset is pt*16 + n
  // ragged tiles: the forward direction's dxp rows t >= the tile's length are zero (lstm_bwd never processes those
  // steps): read through a buffer descriptor at an out-of-range offset -> 0, no bytes moved (~15% of the reads)
  const auto rd0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(dxp), (short)0, (int)(dstride * 2),
                                                     0x00020000);
  auto load = [&](int ks, u16x8_t& b0, u16x8_t& b1, u16x8_t& pp, bool& ok) {
    const int tile = 2 * ks + (q >> 1);
    ok = cval && tile < ntiles && ks < k1;
    const int tl = tile < ntiles ? tile : ntiles - 1;
    const size_t o = (((size_t)tl * L + t) * (NPF + 1) + f) * 16 + half;
    const bool live0 = tlen == nullptr || t < tlen[tl];
    b0 = __builtin_bit_cast(u16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rd0, live0 ? (uint32_t)(o * 2) : 0x80000000u,
                                                                            0, 0));
    b1 = *reinterpret_cast<const u16x8_t*>(dxp + dstride + o);
    pp = *reinterpret_cast<const u16x8_t*>(posb + (size_t)tl * L * 16 + half);   // ids at t = 0
  };
  u16x8_t nb0, nb1, npp;
  bool nok;
  if (k0 < k1) load(k0, nb0, nb1, npp, nok);
  for (int ks = k0; ks < k1; ++ks) {
    u16x8_t b0 = nb0, b1 = nb1, pp = npp;
    const bool ok = nok;
    load(ks + 1, nb0, nb1, npp, nok);   // clamped addresses past the chunk: loaded, never used
    if (!ok) b0 = b1 = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    // pair bits m = (1 << tile(o_2w)) | (1 << (16 + tile(o_2w+1))) for sequences whose offset lands on
    // row n (15 = no hit, never a tile index); tile pt's packed bf16 pair = ((m >> pt) & 0x10001) * 0x3F80
    uint32_t m[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t o0 = ((uint32_t)pp[2 * w] >> sh) & 0xFF, o1 = ((uint32_t)pp[2 * w + 1] >> sh) & 0xFF;
      const uint32_t h0 = (o0 & 15) == (uint32_t)n ? (o0 >> 4) : 15u;
      const uint32_t h1 = (o1 & 15) == (uint32_t)n ? (o1 >> 4) : 15u;
      m[w] = (1u << h0) | (1u << (16 + h1));
    }
#pragma unroll
    for (int pt = 0; pt < NRT; ++pt) {
      uint32_t wv[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) wv[w] = __umul24((m[w] >> pt) & 0x10001u, 0x3F80u);
      u16x8_t a;
      __builtin_memcpy(&a, wv, 16);
      acc[pt] = mfma_bf16(a, b0, acc[pt]);
      acc[pt] = mfma_bf16(a, b1, acc[pt]);
    }
  }
  // D[row = 4q + r][col = n] of tile pt = (offset pt*16 + 4q + r, column nt*16 + n)
  float* g = gpart + ((size_t)blockIdx.y * 2 + tb) * (NRT * 16) * (NT * 16);
#pragma unroll
  for (int pt = 0; pt < NRT; ++pt)
#pragma unroll
    for (int r = 0; r < 4; ++r) g[(size_t)(pt * 16 + 4 * q + r) * (NT * 16) + nt * 16 + n] = acc[pt][r];
}

// out[tb][p][c] = sum_chunk sum_t gpart[chunk][tb][p - t][t * PD + c]   (one workgroup per output)
__global__ __launch_bounds__(256) void pos_shift_finish_kernel(const float* __restrict__ gpart, int nchunk, int L,
                                                               int PD, int rows, float* __restrict__ out) {
  __shared__ float red[4];
  const int P2 = 2 * L, NT = (L * PD + 15) / 16;
  const int id = blockIdx.x;   // (tb * P2 + p) * PD + c
  const int c = id % PD, p = (id / PD) % P2, tb = id / (PD * P2);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tlo = max(0, p - rows + 1), thi = min(L - 1, p);   // 0 <= p - t < rows
  const int nt_ = thi >= tlo ? thi - tlo + 1 : 0;
  float acc = 0.f;
  for (int i = threadIdx.x; i < nchunk * nt_; i += 256) {
    const int ch = i / nt_, t = tlo + (i - ch * nt_);
    acc += gpart[(((size_t)ch * 2 + tb) * rows + (p - t)) * (NT * 16) + t * PD + c];
  }
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[id] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
namespace ina {



// mirrors the kernel's LDS carve (lstm_bwd_kernel)
size_t lstm_bwd_lds_bytes(int U, int NX, bool bf16, int L, int PD, bool xd) {
  const int KPL = bf16 ? 8 : 1;
  const int U4 = U / 4, NSLOT = U4 + NX;
  const int NA = U4 * ((NSLOT + KPL - 1) / KPL) * 64;
  const int NA2 = ((NSLOT + 3) / 4) * ((4 * U4 + KPL - 1) / KPL) * 64;
  const int fragb = bf16 ? 16 : 4;
  const int GT = (4 * U + 15) / 16;
  const int FTMAX = (4 * NX + U + 1 + 15) / 16;
  const int RS = bf16 ? 40 : 36;
  size_t off = (size_t)(NA + NA2) * fragb + 4 * U * 4;
  off = (off + 15) & ~(size_t)15;
  size_t xp = (size_t)4 * (GT * 16 + FTMAX * 16) * RS * (bf16 ? 2 : 4);
  const size_t red = (size_t)4 * U * (4 * NX + U + 1) * 4;
  off += xp > red ? xp : red;
  off = (off + 15) & ~(size_t)15;
  if (!bf16) off += (size_t)2 * 2 * L * PD * 4;   // block pos tables (bf16 mode: pos_grad_kernel)
  if (xd) off = ((off + 15) & ~(size_t)15) + xd_table_bytes(L);   // direct-x position tables
  return off;
}

template <int U, int NX, bool BF16>
static int launch_fwd_t(const LstmArgs& a, hipStream_t st) {
  using frag = typename FragT<BF16>::type;
  using elem = typename FragT<BF16>::elem;
  const int ntiles = (a.S + 15) / 16;
  dim3 grid((ntiles + 3) / 4, 2);
  constexpr bool XDC = BF16 && NX == 4;   // the direct-x kernels exist for 4 x slots per lane only
  const bool xd = XDC && a.xd;
  if (a.xd && !xd) return -1;
  size_t lds = xd ? xd_table_bytes(a.L) : (BF16 ? 0 : (size_t)4 * 16 * a.L * sizeof(int2));   // fp32: token ids
  const bool store = a.hraw != nullptr && a.cst != nullptr;
  // bf16: the keep bits come from x_gather_kernel (x_gather must run first); fp32 hashes them here
  const bool drop = a.drop && !BF16;
  auto kern = drop ? (store ? lstm_fwd_kernel<U, NX, BF16, !BF16, true> : lstm_fwd_kernel<U, NX, BF16, !BF16, false>)
                   : (store ? lstm_fwd_kernel<U, NX, BF16, false, true> : lstm_fwd_kernel<U, NX, BF16, false, false>);
  if (BF16 && a.slen)   // sequence_length semantics (lstm_skip_padding)
    kern = store ? lstm_fwd_kernel<U, NX, BF16, false, true, BF16> : lstm_fwd_kernel<U, NX, BF16, false, false, BF16>;
  if (xd)
    kern = a.slen ? (store ? lstm_fwd_kernel<U, NX, BF16, false, true, BF16, XDC>
                           : lstm_fwd_kernel<U, NX, BF16, false, false, BF16, XDC>)
                  : (store ? lstm_fwd_kernel<U, NX, BF16, false, true, false, XDC>
                           : lstm_fwd_kernel<U, NX, BF16, false, false, false, XDC>);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, a.inst, a.S, a.word, a.pos1, a.pos2, a.L, a.wemb, a.E,
                     a.p1emb, a.p2emb, a.PD, (const frag*)a.apack, a.bias, (elem*)a.hraw,
                     (typename CT<BF16>::type*)a.cst, (elem*)a.hdrop, a.dmask, a.seed, a.thr, a.inv_kp, a.drop, a.seed_dev,
                     (const unsigned short*)(xd ? a.xdtab : a.xg), BF16 ? a.tlen : nullptr, BF16 ? a.slen : nullptr,
                     (const unsigned short*)a.wrows, a.wbytes);
  INA_CHECK_LAUNCH();
  return 0;
}

template <int U, int NX, bool BF16>
static int launch_bwd_t(const LstmArgs& a, hipStream_t st) {
  using frag = typename FragT<BF16>::type;
  using elem = typename FragT<BF16>::elem;
  dim3 grid(a.bwd_blocks, 2);
  // bf16 + lane-layout dH (rec_attn_bwd, premasked): the lean PM step
  const bool pm = BF16 && a.dh_lane;
  constexpr bool XDC = BF16 && NX == 4;   // the direct-x kernels exist for 4 x slots per lane only
  const bool xd = XDC && pm && a.xd;
  if (a.xd && !xd) return -1;
  size_t lds = lstm_bwd_lds_bytes(U, NX, BF16, a.L, a.PD, xd);
  constexpr bool P = BF16;   // the PM / XD kernels exist in bf16 mode only
  auto kfn = pm ? (a.dwemb ? lstm_bwd_kernel<U, NX, BF16, true, P> : lstm_bwd_kernel<U, NX, BF16, false, P>)
                : (a.dwemb ? lstm_bwd_kernel<U, NX, BF16, true, false> : lstm_bwd_kernel<U, NX, BF16, false, false>);
  if (xd) kfn = a.dwemb ? lstm_bwd_kernel<U, NX, BF16, true, P, XDC> : lstm_bwd_kernel<U, NX, BF16, false, P, XDC>;
  static bool attr_set = false;
  if (!attr_set) {
    for (auto f : {lstm_bwd_kernel<U, NX, BF16, true, false>, lstm_bwd_kernel<U, NX, BF16, false, false>,
                   lstm_bwd_kernel<U, NX, BF16, true, P>, lstm_bwd_kernel<U, NX, BF16, false, P>,
                   lstm_bwd_kernel<U, NX, BF16, true, P, XDC>, lstm_bwd_kernel<U, NX, BF16, false, P, XDC>})
      hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(256), lds, st, a.inst, a.S, a.word, a.pos1, a.pos2, a.L, a.wemb, a.E,
                     a.p1emb, a.p2emb, a.PD, (const frag*)a.apack, (const frag*)a.a2pack, a.bias,
                     (const elem*)a.hraw, (const typename CT<BF16>::type*)a.cst, (const elem*)a.dH, a.dw_slab, a.dpos_slab, a.dwemb, a.dmask, a.seed, a.thr, a.inv_kp,
                     a.drop, (unsigned short*)a.dxp, (const unsigned short*)(xd ? a.xdtab : a.xg), a.dh_lane,
                     pm ? a.tlen : nullptr, pm ? a.slen : nullptr, a.wblank, (const unsigned short*)a.wrows,
                     a.wbytes);
  INA_CHECK_LAUNCH();
  return 0;
}

#define INA_LSTM_DISPATCH(FN)                                                        \
  if (bf16) {                                                                        \
    if (U == 20 && NX == 4) return FN<20, 4, true>(a, st);                           \
    if (U == 20 && NX == 16) return FN<20, 16, true>(a, st);                         \
    if (U == 32 && NX == 4) return FN<32, 4, true>(a, st);                           \
    if (U == 32 && NX == 16) return FN<32, 16, true>(a, st);                         \
    if (U == 8 && NX == 4) return FN<8, 4, true>(a, st);                             \
  } else {                                                                           \
    if (U == 20 && NX == 4) return FN<20, 4, false>(a, st);                          \
    if (U == 20 && NX == 16) return FN<20, 16, false>(a, st);                        \
    if (U == 32 && NX == 4) return FN<32, 4, false>(a, st);                          \
    if (U == 32 && NX == 16) return FN<32, 16, false>(a, st);                        \
    if (U == 8 && NX == 4) return FN<8, 4, false>(a, st);                            \
  }                                                                                  \
  return -1;

// Resident workgroups of the persistent backward PER DIRECTION (occupancy x CUs / 2): the default grid,
// so all of the recurrence's waves run in one round (a 512-per-direction grid at 2 workgroups per CU
// ran two rounds of 3-4 tile groups per workgroup: critical path 8 groups for 6.25 of work).
template <int U, int NX, bool BF16>
static int bwd_resident_t(int L, int PD) {
  static int cached[2][129][9];
  const int Lc = L < 128 ? L : 128, Pc = PD < 8 ? PD : 8;
  int& c = cached[BF16][Lc][Pc];
  if (c > 0) return c;
  const size_t lds = lstm_bwd_lds_bytes(U, NX, BF16, L, PD);
  (void)hipFuncSetAttribute((const void*)lstm_bwd_kernel<U, NX, BF16, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_bwd_kernel<U, NX, BF16, false>, 256, lds) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  c = per_cu * cus / 2;
  return c;
}
int lstm_bwd_resident_blocks(int U, int NX, bool bf16, int L, int PD) {
#define INA_BR(UV, NV)                                                     \
  if (U == UV && NX == NV) return bf16 ? bwd_resident_t<UV, NV, true>(L, PD) : bwd_resident_t<UV, NV, false>(L, PD);
  INA_BR(20, 4) INA_BR(20, 16) INA_BR(32, 4) INA_BR(32, 16) INA_BR(8, 4)
#undef INA_BR
  return 0;
}

int lstm_fwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st) { INA_LSTM_DISPATCH(launch_fwd_t) }
int lstm_bwd(const LstmArgs& a, int U, int NX, bool bf16, hipStream_t st) { INA_LSTM_DISPATCH(launch_bwd_t) }

int pos_grad(const LstmArgs& a, int blocks, float* slab, hipStream_t st) {
  const int P2 = 2 * a.L;
  dim3 grid(blocks), block(256);
  const auto* dxp = (const unsigned short*)a.dxp;
  if (P2 <= 48) {
    hipLaunchKernelGGL(pos_grad_kernel<3>, grid, block, 0, st, dxp, a.posb, a.S, a.L, a.PD, slab);
  } else if (P2 <= 80) {
    hipLaunchKernelGGL(pos_grad_kernel<5>, grid, block, 0, st, dxp, a.posb, a.S, a.L, a.PD, slab);
  } else if (P2 <= 128) {
    hipLaunchKernelGGL(pos_grad_kernel<8>, grid, block, 0, st, dxp, a.posb, a.S, a.L, a.PD, slab);
  } else {
    return -1;
  }
  INA_CHECK_LAUNCH();
  return 0;
}

size_t pos_shift_workspace_floats(int S, int L, int PD, int* nchunk, int* kps) {
  const int ntiles = (S + 15) / 16, ksteps = (ntiles + 1) / 2;
  const int NT = (L * PD + 15) / 16, NRT = (L + 1 + 15) / 16 <= 3 ? 3 : 5;
  int nc = (4096 + 2 * NT - 1) / (2 * NT);      // ~4096 waves in flight
  nc = nc < 1 ? 1 : (nc > ksteps ? ksteps : nc);
  const int k = (ksteps + nc - 1) / nc;
  nc = (ksteps + k - 1) / k;
  if (nchunk) *nchunk = nc;
  if (kps) *kps = k;
  return (size_t)nc * 2 * NRT * 16 * NT * 16;
}

int pos_grad_shift(const LstmArgs& a, float* gpart, float* out, hipStream_t st) {
  int nchunk = 0, kps = 0;
  pos_shift_workspace_floats(a.S, a.L, a.PD, &nchunk, &kps);
  const int NT = (a.L * a.PD + 15) / 16, NRT = (a.L + 1 + 15) / 16;
  if (NRT > 5 || a.S <= 0) return -1;
  const auto* dxp = (const unsigned short*)a.dxp;
  dim3 grid((2 * NT + 3) / 4, nchunk), block(256);
  if (NRT <= 3)
    hipLaunchKernelGGL(pos_shift_gemm_kernel<3>, grid, block, 0, st, dxp, a.posb, a.S, a.L, a.PD, kps, gpart, a.tlen);
  else
    hipLaunchKernelGGL(pos_shift_gemm_kernel<5>, grid, block, 0, st, dxp, a.posb, a.S, a.L, a.PD, kps, gpart, a.tlen);
  INA_CHECK_LAUNCH();
  const int rows = (NRT <= 3 ? 3 : 5) * 16;
  hipLaunchKernelGGL(pos_shift_finish_kernel, dim3(2 * 2 * a.L * a.PD), dim3(256), 0, st, gpart, nchunk, a.L, a.PD,
                     rows, out);
  INA_CHECK_LAUNCH();
  return 0;
}

int h_natural(const void* rec, const unsigned char* dmask, float inv_kp, int S, int L, int U, void* hnat,
              hipStream_t st) {
  const int ntiles = (S + 15) / 16;
  if (ntiles <= 0) return 0;
  const size_t lds = (((size_t)2 * L * (U / 4) * 64 * sizeof(unsigned short) + 1023) & ~(size_t)1023) +
                     (dmask ? (((size_t)2 * L * 64 + 1023) & ~(size_t)1023) : 0);
  const auto* hl = rec;
  if (lds > 160 * 1024) return -1;
  const auto* in = (const unsigned short*)hl;
  auto* out = (unsigned short*)hnat;
#define INA_HN(UV)                                                                                     \
  if (U == UV) {                                                                                       \
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)h_natural_kernel<UV>,                        \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
    hipLaunchKernelGGL(h_natural_kernel<UV>, dim3(ntiles), dim3(256), lds, st, in, dmask, L, inv_kp, out); \
    INA_CHECK_LAUNCH();                                                                                \
    return 0;                                                                                          \
  }
  INA_HN(20)
  INA_HN(32)
  INA_HN(8)
#undef INA_HN
  return -1;
}

int x_gather(const LstmArgs& a, int U, int NX, hipStream_t st) {
  const int ntiles = (a.S + 15) / 16;
  if (ntiles <= 0) return 0;
  auto* xg = (unsigned short*)a.xg;
  auto* posb = const_cast<unsigned short*>(a.posb);
  dim3 grid(ntiles, (a.L + XG_T * XG_C - 1) / (XG_T * XG_C));
  if (2 * a.L * a.PD > 128 * 8) return -1;   // pos tables staged in LDS
  const auto* wr16 = (const unsigned short*)a.wrows;
  // one workgroup per tile (capped grid-stride grids measured slower: the direct-x gather is bound by its
  // keep-bit hash, not by workgroup launches -- profiles/r4_xgather_grid)
  if (a.xd && !a.drop) {
    hipLaunchKernelGGL(xd_ids_kernel, dim3((ntiles * 16 + 255) / 256), dim3(256), 0, st, a.inst, a.S, a.pos1, a.pos2,
                       a.L, a.E, a.PD, a.p1emb, a.p2emb, posb, (unsigned short*)a.xdtab);
    INA_CHECK_LAUNCH();
    return 0;
  }
#define INA_XG_LAUNCH(NXV, DIR, ...)                                                                     \
  hipLaunchKernelGGL((x_gather_kernel<NXV, DIR, ##__VA_ARGS__>), grid, dim3(256), 0, st, a.inst, a.S, a.word, a.pos1, a.pos2, a.L, \
                     a.wemb, wr16, a.E, a.p1emb, a.p2emb, a.PD, xg, posb, a.drop ? a.dmask : nullptr, U, a.seed, \
                     a.seed_dev, a.thr, a.perm, a.xd ? (unsigned short*)a.xdtab : nullptr, a.tlen)
  if (NX == 4 && a.wrows && U == 20 && a.E == 5 && a.PD == 5)
    INA_XG_LAUNCH(4, true, 20, 5, 5);
  else if (NX == 4 && a.wrows)
    INA_XG_LAUNCH(4, true);
  else if (NX == 4)
    INA_XG_LAUNCH(4, false);
  else if (NX == 16 && a.wrows)
    INA_XG_LAUNCH(16, true);
  else if (NX == 16)
    INA_XG_LAUNCH(16, false);
  else
    return -1;
#undef INA_XG_LAUNCH
  INA_CHECK_LAUNCH();
  return 0;
}

bool lstm_supported(int U, int NX) {
  return (U == 20 || U == 32 || U == 8) && (NX == 4 || NX == 16);
}

}  // namespace ina
