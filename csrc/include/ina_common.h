// Shared device helpers for the Induction-Network gfx950 kernels.
//
// Conventions used by every kernel in csrc/kernels:
//  * wave = 64 lanes; MFMA v_mfma_f32_16x16x32_bf16 (bf16 path) or v_mfma_f32_16x16x4_f32
//    (fp32 path).  For both, lane l holds A[row = l&15][k = KPL*(l>>4) + j] and
//    B[k = KPL*(l>>4) + j][col = l&15] (j < KPL, KPL = 8 for bf16, 1 for fp32) and the
//    accumulator C[row = 4*(l>>4) + r][col = l&15], r = 0..3.
//  * "lane group" q = l >> 4 (0..3); "lane column" n = l & 15.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define INA_DEVICE __device__ __forceinline__

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

namespace ina {

// ------------------------------------------------------------------ bf16 bits
INA_DEVICE unsigned short f2bf(float f) {
  __bf16 h = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32 on gfx950)
  return __builtin_bit_cast(unsigned short, h);
}
INA_DEVICE float bf2f(unsigned short b) { return __builtin_bit_cast(float, ((uint32_t)b) << 16); }
INA_DEVICE float round_bf(float f) { return bf2f(f2bf(f)); }

// ------------------------------------------------------------------ MFMA
INA_DEVICE f32x4_t mfma_bf16(const u16x8_t& a, const u16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
INA_DEVICE f32x4_t mfma_f32(float a, float b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// v_mfma_f32_16x16x16_bf16: lane l holds A[row l&15][k = 4(l>>4) + j], B[k = 4(l>>4) + j][col l&15], j < 4
INA_DEVICE f32x4_t mfma16_bf16(const s16x4_t& a, const s16x4_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// ds_read_b64_tr_b16 (gfx950 hardware transpose, EXEC must be all ones).  From a row-major LDS
// image [k rows][cols] of 16-bit values, each lane passing the address of
//   row 4 (l>>4) + ((l&15)>>2), column c0 + 4 (l&3)       (8-byte aligned)
// returns the 16x16x16 operand fragment {image[4(l>>4) + j][c0 + (l&15)], j < 4}: a [k][col] block
// read as a B operand, or as the A operand of the transposed block.
INA_DEVICE s16x4_t tr_read(const unsigned short* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)lds_addr);
}
// 16x16x32 operand fragment from a row-major LDS image [k rows][cols] (two ds_read_b64_tr_b16):
// element j of lane (q = l >> 4, n = l & 15) = image[8 q + j][c0 + n] -- the B operand B[k][c0 + n], or
// the A operand A[c0 + n][k] of the transposed block.  stride (elements) * 2 and c0 * 2 must be 8-byte
// multiples; EXEC must be all ones.
INA_DEVICE u16x8_t tr_read8(const unsigned short* img, int stride, int c0, int q, int n) {
  const s16x4_t lo = tr_read(img + (8 * q + (n >> 2)) * stride + c0 + 4 * (n & 3));
  const s16x4_t hi = tr_read(img + (8 * q + 4 + (n >> 2)) * stride + c0 + 4 * (n & 3));
  return u16x8_t{(unsigned short)lo[0], (unsigned short)lo[1], (unsigned short)lo[2], (unsigned short)lo[3],
                 (unsigned short)hi[0], (unsigned short)hi[1], (unsigned short)hi[2], (unsigned short)hi[3]};
}

// LDS-DMA of 16 B per lane (lane-linear from the wave-uniform LDS byte address lds_dst) as inline asm
// (cdna_hip_programming.md 5.7 recipe: M0 saved / set / restored in the statement).  hipcc does not see it,
// so it does not make later ds_read_b64_tr_b16 wait for it (with the builtin it cannot prove the transposed
// reads disjoint from the DMA target and drains vmcnt before every one); the caller counts the completion
// (s_waitcnt vmcnt + a workgroup barrier before the data is read).
INA_DEVICE void glds16_asm(const void* gsrc_lane, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc_lane), "s"(lds_dst)
               : "memory");
}
// 32-bit LDS byte address of a __shared__ pointer
INA_DEVICE uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
}

// order this wave's LDS accesses without a memory fence: a wave's own LDS operations execute in
// order in hardware, and a fence would also wait for every in-flight global load (vmcnt(0))
INA_DEVICE void lds_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ math
// v_rcp_f32 (1 ulp) instead of the IEEE division sequence (div_scale/div_fmas/div_fixup): the
// activations sit on the recurrence's dependency chain, so instruction latency is what matters.
INA_DEVICE float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
INA_DEVICE float sigmoidf_(float x) { return fast_rcp(1.0f + __expf(-x)); }
INA_DEVICE float tanhf_(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1); saturates cleanly at +-1, abs err ~2e-7
  const float e = __expf(2.0f * x);
  return 1.0f - 2.0f * fast_rcp(e + 1.0f);
}
// Pre-scaled forms: the argument already carries the exp2 range factor, z = log2(e) x (sigmoid)
// resp. z = 2 log2(e) x (tanh).  The LSTM kernels fold these factors into their gate weight rows
// and biases once per kernel, so each activation on the recurrence is v_exp + v_add + v_rcp
// (+ one v_fma for tanh): no per-step range multiply.
constexpr float LOG2E_F = 1.44269504088896341f;
INA_DEVICE float sigmoid_l2(float z) { return fast_rcp(1.0f + __builtin_amdgcn_exp2f(-z)); }
INA_DEVICE float tanh_l2(float z) { return 1.0f - 2.0f * fast_rcp(__builtin_amdgcn_exp2f(z) + 1.0f); }
// r = 1 / (e^{2x} + 1): tanh(x) = 1 - 2 r and 1 - tanh(x)^2 = 4 r (1 - r) (same rounding as tanhf_)
INA_DEVICE float tanh_r(float x) { return fast_rcp(__builtin_amdgcn_exp2f(x * (2.0f * LOG2E_F)) + 1.0f); }
// the same for a 4-vector (the range multiply as two packed v_pk_mul_f32)
INA_DEVICE f32x4_t tanh_r4(f32x4_t x) {
  x *= 2.0f * LOG2E_F;
  f32x4_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = fast_rcp(__builtin_amdgcn_exp2f(x[i]) + 1.0f);
  return r;
}

// ------------------------------------------------------------------ RNG
// Counter-based hash; bit-identical to models/reference.py::hash_u32.
INA_DEVICE uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x68E31DA4u;
  x ^= x >> 16;
  return x;
}
// Dropout: keep element `idx` (flat (seq*L + t)*U + unit) of direction `dir` iff
// mix(idx * C1 + salt(seed, dir)) < thr.  Bit-identical to models/reference.py::dropout_keep_mask.
INA_DEVICE uint32_t dropout_salt(uint32_t seed, uint32_t dir) {
  return seed * 0x2545F491u + dir * 0x3C6EF372u + 0x1234567u;
}
INA_DEVICE bool dropout_keep_salted(uint32_t salt, uint32_t idx, uint32_t thr) {
  uint32_t x = idx * 0x6C8E9CF5u + salt;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x < thr;
}
INA_DEVICE bool dropout_keep(uint32_t seed, uint32_t dir, uint32_t idx, uint32_t thr) {
  return dropout_keep_salted(dropout_salt(seed, dir), idx, thr);
}
// LSTM output dropout (DropoutWrapper): ONE hash per pair of adjacent units.  Element e (flat
// (seq*L + t)*U + unit, U even) keeps iff 16-bit half (e & 1) of mix(e >> 1) is < thr >> 16
// (keep rate floor(kp * 65536) / 65536).  Bit-identical to models/reference.py::dropout_keep_mask.
INA_DEVICE uint32_t dropout_mix(uint32_t salt, uint32_t pidx) {
  uint32_t x = pidx * 0x6C8E9CF5u + salt;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x;
}
INA_DEVICE bool lstm_keep(uint32_t salt, uint32_t e, uint32_t thr) {
  const uint32_t x = dropout_mix(salt, e >> 1);
  return ((e & 1u) ? (x >> 16) : (x & 0xFFFFu)) < (thr >> 16);
}

// ------------------------------------------------------------------ reductions
// Cross-lane data movement without the LDS pipe: __shfl_xor lowers to ds_bpermute_b32 (an LDS
// instruction with tens of cycles of latency plus an address VGPR); these use DPP lane permutes
// inside a 16-lane row (folded into the v_add / v_max) and the gfx950 v_permlane16/32_swap row
// exchanges across rows.  Every step combines symmetric pairs, so all lanes of the reduced group
// end with bitwise the same value; the order is fixed (deterministic), not the xor-butterfly order.
namespace dpp {
constexpr int QUAD_XOR1 = 0xB1;         // quad_perm:[1,0,3,2]
constexpr int QUAD_XOR2 = 0x4E;         // quad_perm:[2,3,0,1]
constexpr int ROW_HALF_MIRROR = 0x141;  // lane i <- 7 - i within each 8
constexpr int ROW_MIRROR = 0x140;       // lane i <- 15 - i within each 16
template <int CTRL>
INA_DEVICE float mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// permlane16_swap(x, x) -> (rows 0,0,2,2 ; rows 1,1,3,3); permlane32_swap(x, x) -> (lo,lo ; hi,hi)
INA_DEVICE void swap16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}
INA_DEVICE void swap32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                  false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}
}  // namespace dpp

// sum over the 16 lanes that share a lane group (same l>>4)
INA_DEVICE float group16_sum(float v) {
  v += dpp::mov<dpp::QUAD_XOR1>(v);
  v += dpp::mov<dpp::QUAD_XOR2>(v);
  v += dpp::mov<dpp::ROW_HALF_MIRROR>(v);
  v += dpp::mov<dpp::ROW_MIRROR>(v);
  return v;
}
INA_DEVICE float group16_max(float v) {
  v = fmaxf(v, dpp::mov<dpp::QUAD_XOR1>(v));
  v = fmaxf(v, dpp::mov<dpp::QUAD_XOR2>(v));
  v = fmaxf(v, dpp::mov<dpp::ROW_HALF_MIRROR>(v));
  v = fmaxf(v, dpp::mov<dpp::ROW_MIRROR>(v));
  return v;
}
// sum over the 4 lane groups (lanes n, n+16, n+32, n+48)
INA_DEVICE float cross_group_sum(float v) {
  float a, b;
  dpp::swap16(v, a, b);
  dpp::swap32(a + b, a, b);
  return a + b;
}
INA_DEVICE float cross_group_max(float v) {
  float a, b;
  dpp::swap16(v, a, b);
  dpp::swap32(fmaxf(a, b), a, b);
  return fmaxf(a, b);
}
INA_DEVICE float wave_sum(float v) { return cross_group_sum(group16_sum(v)); }

// Store widening: lane group fq holds X = columns 4 fq .. 4 fq + 3 of tile nt = 2h and Y = columns 16 + 4 fq ..
// of tile 2h + 1 (4 bf16 each, one row).  permlane32_swap (upper half of X <-> lower half of Y) then
// permlane16_swap (odd 16-lane rows of X <-> even rows of Y) leave lane group fq with columns 8 fq .. 8 fq + 7
// as (X, Y): one 16-byte store per lane, 16 rows x 64 B per instruction instead of two of 16 rows x 32 B
// (the C write of a short-K GEMM is store-issue bound: cdna_hip_programming.md T21; used by gemm.hip and
// attn_wide.hip).  Semantics checked by tools/lds_probe/permlane_probe.hip.
INA_DEVICE void widen(uint2& X, uint2& Y) {
  auto r = __builtin_amdgcn_permlane32_swap(X.x, Y.x, false, false);
  X.x = r[0];
  Y.x = r[1];
  r = __builtin_amdgcn_permlane32_swap(X.y, Y.y, false, false);
  X.y = r[0];
  Y.y = r[1];
  r = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
  X.x = r[0];
  Y.x = r[1];
  r = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
  X.y = r[0];
  Y.y = r[1];
}

// The inverse exchange (each swap is an involution): a 16-byte row chunk loaded in the widened layout (lane
// group fq: columns 8 fq .. 8 fq + 7) back to the accumulator layout (X: tile 2h columns 4 fq .., Y: tile 2h + 1).
// (The widening is applied to VALU results only: a permlane swap reading an MFMA accumulator directly gets no
// MFMA -> VALU wait states from hipcc and read stale values.)
INA_DEVICE void unwiden(uint2& X, uint2& Y) {
  auto r = __builtin_amdgcn_permlane16_swap(X.x, Y.x, false, false);
  X.x = r[0];
  Y.x = r[1];
  r = __builtin_amdgcn_permlane16_swap(X.y, Y.y, false, false);
  X.y = r[0];
  Y.y = r[1];
  r = __builtin_amdgcn_permlane32_swap(X.x, Y.x, false, false);
  X.x = r[0];
  Y.x = r[1];
  r = __builtin_amdgcn_permlane32_swap(X.y, Y.y, false, false);
  X.y = r[0];
  Y.y = r[1];
}

INA_DEVICE float wave_max(float v) { return cross_group_max(group16_max(v)); }

// Deterministic workgroup reduction: the waves add their contributions into a shared LDS buffer one
// after another (wave 0 first), so the fp32 summation order never depends on scheduling (LDS float
// atomics would).  body() does plain read-add-writes; within one wave every lane must own distinct
// addresses.  Must be reached by every thread of the workgroup.
template <class F>
INA_DEVICE void ordered_wave_accumulate(int wave, int nwaves, F&& body) {
  for (int w = 0; w < nwaves; ++w) {
    if (wave == w) body();
    __syncthreads();
  }
}

}  // namespace ina

#define INA_CHECK_LAUNCH()                                                        \
  do {                                                                            \
    hipError_t e__ = hipGetLastError();                                           \
    if (e__ != hipSuccess) return (int)e__;                                       \
  } while (0)
