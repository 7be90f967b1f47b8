// Fused neural-tensor-layer relation module (K7 + K8 of SURVEY 2.3), bf16 MFMA, fp32 accumulate.
//
// Reference (model/layer_module.py:8-47, model/graph.py:81-86):
//   for s in 0..h-1:  S_s = (C @ M[:,:,s]) @ Q^T          [N, NQ]
//   V = relu(concat_s(S_s)^T)  with column index s*N + c   [NQ, h*N]
//   probs = sigmoid(V @ w + b),  w [h*N, N], b [N]        ("reference" head)
// "paper" head (paper Eq.11): probs[q, c] = sigmoid(sum_s w_s relu(T[q, s, c]) + b).
//
// One wave per episode; the 200 tiny GEMMs of the reference become one chained MFMA pipeline per
// slice pair, entirely in registers:
//   P_s^T[b, c] = M_s^T[b, a] C^T[a, c]                          (M pre-packed per step)
//   T_s[c, q]   = P_s[c, b] Q^T[b, q]      P^T accumulator reused as the A operand
//   logits[q,c']+= relu(T)[(s,c), q]^T w[(s,c), c']   relu(T) accumulators of TWO slices form one
//                                                      32-deep K step
// An accumulator tile X (rows 4*(l>>4)+r, column l&15) used as an operand contracts over X's ROW
// index; two tiles are paired into one K=32 fragment with k = 8q + j <-> row 16*(j>>2) + 4q + (j&3)
// ("kmap32").  Every memory operand that meets such a fragment is packed with the same map.
// The backward recomputes P/T and produces dC, dQ (registers, summed over slices), the per-episode
// dw contribution and dP (bf16, for the dM = C^T dP reduction GEMM across episodes).
//
// A workgroup is 8 waves = 8 episodes; the packed M / w fragments of each slice pair are staged ONCE
// per workgroup into LDS (double buffered, one barrier per pair) and shared by the 8 episodes, so the
// L2 traffic for M is 1/8 of a wave-per-episode design (which measured 76 % SQ_WAIT_ANY).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

INA_DEVICE u16x8_t pack2(const f32x4_t& x0, const f32x4_t& x1) {
  u16x8_t f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = f2bf(x0[j]);
    f[4 + j] = f2bf(x1[j]);
  }
  return f;
}
INA_DEVICE f32x4_t relu4(const f32x4_t& x) {
  return f32x4_t{fmaxf(x[0], 0.f), fmaxf(x[1], 0.f), fmaxf(x[2], 0.f), fmaxf(x[3], 0.f)};
}
INA_DEVICE int kmap32(int q, int j) { return 16 * (j >> 2) + 4 * q + (j & 3); }
// Unconditional load from a clamped index, zero outside: a lane-dependent branch around each load
// made hipcc wait vmcnt(0) per element (60-400 serialized L2 round trips in the prologues).
// (multiply by 0/1 rather than select: a select lets LLVM sink the load back under a branch)
INA_DEVICE float ldz(const float* __restrict__ p, bool ok, long idx) {
  return p[ok ? idx : 0] * (ok ? 1.f : 0.f);
}
// 4 consecutive floats p[idx .. idx + 3] (idx % 4 == 0) -> bf16 elements j0 .. j0 + 3 of f (zeros if !ok)
INA_DEVICE void ld4bf(const float* __restrict__ p, bool ok, long idx, u16x8_t& f, int j0) {
  const float4 v = *reinterpret_cast<const float4*>(p + (ok ? idx : 0));
  const float z = ok ? 1.f : 0.f;
  f[j0] = f2bf(v.x * z);
  f[j0 + 1] = f2bf(v.y * z);
  f[j0 + 2] = f2bf(v.z * z);
  f[j0 + 3] = f2bf(v.w * z);
}
constexpr f32x4_t Z4 = {0.f, 0.f, 0.f, 0.f};

}  // namespace


#ifndef INA_NTN_BWD_LD
#define INA_NTN_BWD_LD 1   // branch-free vectorized prologue loads in ntn_bwd (153 vs 160 us despite 188 B of spills; 0 = the branchy per-element loads)
#endif
#ifndef INA_NTN_TR
#define INA_NTN_TR 1   // ntn_bwd: P^T -> P, T -> T^T and dT -> dT^T through wave-private LDS images read back with
                       // ds_read_b64_tr_b16, instead of recomputing each product in the other layout (37 -> 25 MFMAs
                       // per slice and episode)
#endif
#ifndef INA_NTN_WAVES
#define INA_NTN_WAVES 8   // episodes (waves) per workgroup sharing one staged copy of the slice packs
// (4 episodes: ntn_bwd 574 -> 641 us with two workgroups per CU -- twice the pack staging -- and 1120 us
// without the waves_per_eu(2) bound, which lets it take 331 registers at one wave per SIMD; tools/gpu_ab_ntn.sh)
#endif
constexpr int NTN_WAVES = INA_NTN_WAVES;
constexpr int NTN_THREADS = NTN_WAVES * 64;

// Stage slice pair p straight into LDS with global_load_lds (16 B / lane, one 1-KiB fragment per wave
// instruction, no staging registers).  Staged pair layout (fragments of 64 lanes x 16 B):
// [mpack: 2*MTH*NKA][m2pack: 2*MTH*NKB (backward only)][w: NSW].  The host pads every packed array to
// an even number of slices, so no lane needs a bounds check.
INA_DEVICE void glds16(const u16x8_t* gsrc_lane, u16x8_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc_lane,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}
template <int MTH, int NSW, bool WITH_M2>
INA_DEVICE void ntn_stage(u16x8_t* buf, int p, const u16x8_t* __restrict__ mpack, const u16x8_t* __restrict__ m2pack,
                          const u16x8_t* __restrict__ wsrc, int w_per_pair) {
  constexpr int NKA = (MTH + 1) / 2, NKB = (MTH + 1) / 2;
  constexpr int F1 = 2 * MTH * NKA, F2 = WITH_M2 ? 2 * MTH * NKB : 0, FR = F1 + F2 + NSW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int f = wave; f < FR; f += NTN_WAVES) {
    const u16x8_t* src;
    if (f < F1)
      src = mpack + ((long)2 * p * MTH * NKA + f) * 64;
    else if (f < F1 + F2)
      src = m2pack + ((long)2 * p * MTH * NKB + (f - F1)) * 64;
    else
      src = wsrc + ((long)p * w_per_pair + (f - F1 - F2)) * 64;
    glds16(src + lane, buf + f * 64);
  }
}
INA_DEVICE void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------------------------------------
template <int MTH, int QT, bool PAPER>
__global__ __launch_bounds__(NTN_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void ntn_fwd_kernel(const float* __restrict__ cls, const float* __restrict__ e,
                                                              int E, int N, int K, int Q, int H, int h,
                                                              const u16x8_t* __restrict__ mpack,
                                                              const u16x8_t* __restrict__ wpack,
                                                              const float* __restrict__ wvec,
                                                              const float* __restrict__ bias, float* __restrict__ probs,
                                                              float* __restrict__ part) {
  constexpr int NKA = (MTH + 1) / 2;  // K steps over a (32 each)
  constexpr int NKB = (MTH + 1) / 2;  // K steps over b (pairs of accumulator tiles)
  constexpr int NSW = PAPER ? 0 : 1;
  constexpr int FR = 2 * MTH * NKA + NSW;
  extern __shared__ __attribute__((aligned(16))) u16x8_t ntn_lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15, wave = threadIdx.x >> 6;
  const int NQ = N * Q;
  const int npair = (h + 1) / 2;
  // slice split (small episode batches): workgroup row blockIdx.y takes slice pairs [p0, p1) and writes
  // raw logit partials; ntn_fwd_finish sums them in split order (deterministic)
  const int p0 = (int)((long)npair * blockIdx.y / gridDim.y), p1 = (int)((long)npair * (blockIdx.y + 1) / gridDim.y);
  for (int g = blockIdx.x; g * NTN_WAVES < E; g += gridDim.x) {
    const int ep = g * NTN_WAVES + wave;
    const bool act = ep < E;
    const int epc = act ? ep : E - 1;
    const long rq0 = (long)epc * (N * K + NQ) + N * K;
    // H % 8 == 0 (host check): every 4-feature run is in or out of range as a whole -> float4 loads
    u16x8_t Cf[NKA];
#pragma unroll
    for (int ka = 0; ka < NKA; ++ka)
#pragma unroll
      for (int h4 = 0; h4 < 2; ++h4) {
        const int a = 32 * ka + 8 * q + 4 * h4;
        ld4bf(cls, n < N && a < H, ((long)epc * N + n) * H + a, Cf[ka], 4 * h4);
      }
    u16x8_t Qf[QT][NKB];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int h4 = 0; h4 < 2; ++h4) {   // kmap32: elements 4 h4 .. +3 = features 32 kb + 16 h4 + 4q .. +3
          const int qi = 16 * qt + n, b = 32 * kb + 16 * h4 + 4 * q;
          ld4bf(e, qi < NQ && b < H, (rq0 + qi) * H + b, Qf[qt][kb], 4 * h4);
        }
    f32x4_t Lg[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) Lg[qt] = Z4;
    __syncthreads();  // previous group's readers are done with buffer 0
    ntn_stage<MTH, NSW, false>(ntn_lds, p0, mpack, nullptr, wpack, 1);
    stage_wait();
    __syncthreads();
    for (int p = p0; p < p1; ++p) {
      const u16x8_t* buf = ntn_lds + ((p - p0) & 1) * FR * 64;
      if (p + 1 < p1) ntn_stage<MTH, NSW, false>(ntn_lds + ((p + 1 - p0) & 1) * FR * 64, p + 1, mpack, nullptr, wpack, 1);
      if (act) {
        f32x4_t V[2][QT];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const int s = 2 * p + sl;
          f32x4_t PT[2 * NKB];
#pragma unroll
          for (int mb = 0; mb < 2 * NKB; ++mb) {
            PT[mb] = Z4;
            if (mb < MTH) {
#pragma unroll
              for (int ka = 0; ka < NKA; ++ka)
                PT[mb] = mfma_bf16(buf[((sl * MTH + mb) * NKA + ka) * 64 + lane], Cf[ka], PT[mb]);
            }
          }
          u16x8_t PTf[NKB];
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) PTf[kb] = pack2(PT[2 * kb], PT[2 * kb + 1]);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            f32x4_t T = Z4;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) T = mfma_bf16(PTf[kb], Qf[qt][kb], T);
            if (PAPER) {
              const float ws = s < h ? wvec[s < h ? s : 0] : 0.f;
              const f32x4_t Rl = relu4(T);
#pragma unroll
              for (int r = 0; r < 4; ++r) Lg[qt][r] += ws * Rl[r];
            } else {
              V[sl][qt] = relu4(T);  // zero M for s >= h -> T = 0
            }
          }
        }
        if (!PAPER) {
          const u16x8_t wf = buf[(2 * MTH * NKA) * 64 + lane];
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) Lg[qt] = mfma_bf16(pack2(V[0][qt], V[1][qt]), wf, Lg[qt]);
        }
      }
      stage_wait();
      __syncthreads();
    }
    if (act) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // PAPER: rows c, cols query; reference head: rows query, cols c'
          const int c = PAPER ? 4 * q + r : n, qi = PAPER ? 16 * qt + n : 16 * qt + 4 * q + r;
          if (c < N && qi < NQ) {
            const long o = ((long)ep * NQ + qi) * N + c;
            if (gridDim.y == 1)
              probs[o] = sigmoidf_(Lg[qt][r] + bias[PAPER ? 0 : c]);
            else
              part[(long)blockIdx.y * E * NQ * N + o] = Lg[qt][r];
          }
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Outputs: dcls [E,N,H]; de query rows [S,H]; dp_out bf16 [E*N][h*H] (col s*H + b);
//          dw_slab [ntn_groups(E)][h][N][N] (reference head: the workgroup's 8 episodes summed in fixed wave
//          order through LDS, one slab row per workgroup group) or [E][h] (paper head).
template <int MTH, int QT, bool PAPER>
__global__ __launch_bounds__(NTN_THREADS) __attribute__((amdgpu_waves_per_eu(2))) void ntn_bwd_kernel(
    const float* __restrict__ cls, const float* __restrict__ e, int E, int N, int K, int Q, int H, int h,
    const u16x8_t* __restrict__ mpack, const u16x8_t* __restrict__ m2pack, const u16x8_t* __restrict__ wtpack,
    const float* __restrict__ wvec, const float* __restrict__ dz, float* __restrict__ dcls, float* __restrict__ de,
    unsigned short* __restrict__ dp_out, float* __restrict__ dw_slab, const float* __restrict__ gscale,
    unsigned short* __restrict__ cls_bf, float* __restrict__ pc, float* __restrict__ pq) {
  constexpr int NKA = (MTH + 1) / 2, NKB = (MTH + 1) / 2, KQ = (QT + 1) / 2;
  const float gs = gscale ? gscale[0] : 1.f;   // upstream scale of dz (loss.backward(g))
  constexpr int NSW = PAPER ? 0 : 2;
  constexpr int F1 = 2 * MTH * NKA, F2 = 2 * MTH * NKB;
  constexpr int FR = F1 + F2 + NSW;
  extern __shared__ __attribute__((aligned(16))) u16x8_t ntn_lds[];
  const int lane = threadIdx.x & 63, q = lane >> 4, n = lane & 15, wave = threadIdx.x >> 6;
  const int NQ = N * Q;
  const long hH = (long)h * H;
  const int npair = (h + 1) / 2;
  // slice split: pairs [p0, p1) of workgroup row blockIdx.y; dC / dQ partials -> pc / pq (ntn_bwd_finish)
  const int p0 = (int)((long)npair * blockIdx.y / gridDim.y), p1 = (int)((long)npair * (blockIdx.y + 1) / gridDim.y);
  if (gridDim.y > 1 && blockIdx.y > 0) cls_bf = nullptr;   // one writer of the bf16 class vectors
  for (int g = blockIdx.x; g * NTN_WAVES < E; g += gridDim.x) {
    const int ep = g * NTN_WAVES + wave;
    const bool act = ep < E;
    const int epc = act ? ep : E - 1;
    const long rq0 = (long)epc * (N * K + NQ) + N * K;
    const float* dze = dz + (long)epc * NQ * N;
#if INA_NTN_BWD_LD
    u16x8_t Cf[NKA];
#pragma unroll
    for (int ka = 0; ka < NKA; ++ka)
#pragma unroll
      for (int h4 = 0; h4 < 2; ++h4) {
        const int a = 32 * ka + 8 * q + 4 * h4;
        ld4bf(cls, n < N && a < H, ((long)epc * N + n) * H + a, Cf[ka], 4 * h4);
      }
    if (cls_bf && act && n < N) {
#pragma unroll
      for (int ka = 0; ka < NKA; ++ka) {
        const int a = 32 * ka + 8 * q;
        if (a < H) *reinterpret_cast<u16x8_t*>(cls_bf + ((long)ep * N + n) * H + a) = Cf[ka];
      }
    }
    u16x8_t Qf[QT][NKB];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int h4 = 0; h4 < 2; ++h4) {
          const int qi = 16 * qt + n, b = 32 * kb + 16 * h4 + 4 * q;
          ld4bf(e, qi < NQ && b < H, (rq0 + qi) * H + b, Qf[qt][kb], 4 * h4);
        }
    // Q^T as the A operand over queries: A[i = b][k = query (kmap32)]
    __builtin_amdgcn_sched_barrier(0);   // load groups in turn: bounded registers in flight
    // (TR: natural query order k = q -- the dT^T operand then comes from a row-major LDS image)
    u16x8_t QTf[MTH][KQ];
#pragma unroll
    for (int mb = 0; mb < MTH; ++mb)
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = 16 * mb + n, qi = 32 * kq + (INA_NTN_TR ? 8 * q + j : kmap32(q, j));
          QTf[mb][kq][j] = f2bf(ldz(e, qi < NQ && b < H, (rq0 + qi) * H + b));
        }
    __builtin_amdgcn_sched_barrier(0);
    u16x8_t dzA[QT];           // A[i = query][k = c']
    u16x8_t dzB[KQ];           // B[k = query (kmap32)][j = c']
    f32x4_t dzC[QT], dzR[QT];  // accumulator layouts: dzC rows c / cols query, dzR rows query / cols c
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qi = 16 * qt + n, cp = 8 * q + j;
        dzA[qt][j] = f2bf(gs * ldz(dze, qi < NQ && cp < N, qi * N + cp));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * q + r, qi = 16 * qt + n;
        dzC[qt][r] = gs * ldz(dze, c < N && qi < NQ, qi * N + c);
        const int qr = 16 * qt + 4 * q + r;
        dzR[qt][r] = gs * ldz(dze, n < N && qr < NQ, qr * N + n);
      }
    }
#pragma unroll
    for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qi = 32 * kq + (INA_NTN_TR ? 8 * q + j : kmap32(q, j));
        dzB[kq][j] = f2bf(gs * ldz(dze, qi < NQ && n < N, qi * N + n));
      }
    __builtin_amdgcn_sched_barrier(0);
#else
    static_assert(!INA_NTN_TR, "the LDS-transpose backward needs the vectorized prologue (INA_NTN_BWD_LD)");
    u16x8_t Cf[NKA];
#pragma unroll
    for (int ka = 0; ka < NKA; ++ka)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int a = 32 * ka + 8 * q + j;
        Cf[ka][j] = (n < N && a < H) ? f2bf(cls[((long)epc * N + n) * H + a]) : (unsigned short)0;
        if (cls_bf && act && n < N && a < H) cls_bf[((long)ep * N + n) * H + a] = Cf[ka][j];
      }
    u16x8_t Qf[QT][NKB];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int qi = 16 * qt + n, b = 32 * kb + kmap32(q, j);
          Qf[qt][kb][j] = (qi < NQ && b < H) ? f2bf(e[(rq0 + qi) * H + b]) : (unsigned short)0;
        }
    // Q^T as the A operand over queries: A[i = b][k = query (kmap32)]
    u16x8_t QTf[MTH][KQ];
#pragma unroll
    for (int mb = 0; mb < MTH; ++mb)
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = 16 * mb + n, qi = 32 * kq + kmap32(q, j);
          QTf[mb][kq][j] = (qi < NQ && b < H) ? f2bf(e[(rq0 + qi) * H + b]) : (unsigned short)0;
        }
    u16x8_t dzA[QT];           // A[i = query][k = c']
    u16x8_t dzB[KQ];           // B[k = query (kmap32)][j = c']
    f32x4_t dzC[QT], dzR[QT];  // accumulator layouts: dzC rows c / cols query, dzR rows query / cols c
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qi = 16 * qt + n, cp = 8 * q + j;
        dzA[qt][j] = (qi < NQ && cp < N) ? f2bf(gs * dze[qi * N + cp]) : (unsigned short)0;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * q + r, qi = 16 * qt + n;
        dzC[qt][r] = (c < N && qi < NQ) ? gs * dze[qi * N + c] : 0.f;
        const int qr = 16 * qt + 4 * q + r;
        dzR[qt][r] = (n < N && qr < NQ) ? gs * dze[qr * N + n] : 0.f;
      }
    }
#pragma unroll
    for (int kq = 0; kq < KQ; ++kq)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int qi = 32 * kq + kmap32(q, j);
        dzB[kq][j] = (qi < NQ && n < N) ? f2bf(gs * dze[qi * N + n]) : (unsigned short)0;
      }
#endif
    f32x4_t dCT[MTH], dQT[MTH][QT];
#pragma unroll
    for (int m = 0; m < MTH; ++m) {
      dCT[m] = Z4;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) dQT[m][qt] = Z4;
    }
    // Per-lane store bases of the per-slice dP / dw outputs, chosen once per group: lanes outside
    // the N x N / H ranges point into the trash tail the host allocates past each buffer, so the
    // slice loop's stores are unconditional.  (Guarded stores split the loop into ~15 basic
    // blocks -- exec-mask branches the scheduler cannot move MFMAs across -- and re-derived the
    // 64-bit row offsets with v_mul_lo_u32 per slice.)
    unsigned short* dpb[MTH];
#pragma unroll
    for (int mb = 0; mb < MTH; ++mb) {
      const int b0 = 16 * mb + 4 * q;
      dpb[mb] = dp_out + ((n < N && b0 < H) ? ((long)epc * N + n) * hH + b0 : (long)E * N * hH);
    }
    // reference head dw: per (pair parity, wave, slice) an [N*N + 1] LDS slot (the last entry takes the
    // lanes outside N x N); summed over the group's waves in fixed order one pair later (flush_dw)
    const int NN1 = N * N + 1;
    float* const dwl = reinterpret_cast<float*>(ntn_lds + 2 * FR * 64);
    // TR: wave-private bf16 images (after the dw slots): I_P [32 rows (slice, class)][PS] = the pair's P^T
    // transposed; I_V / I_dT [32 KQ rows (query)][VS] = relu(T) / dT with the queries on the rows
    constexpr int PS = 16 * MTH + 4, VS = 20, IPN = 32 * PS, IVN = 32 * KQ * VS;
    // (byte offset arithmetic on the __shared__ pointer: a uintptr_t round trip would turn these accesses
    // into FLAT instructions)
    unsigned short* const imgP =
        reinterpret_cast<unsigned short*>(reinterpret_cast<unsigned char*>(dwl) +
                                          (((PAPER ? 0 : 2 * NTN_WAVES * 2 * NN1) * 4 + 15) & ~15)) +
        (size_t)wave * (IPN + 2 * IVN);
    unsigned short* const imgV = imgP + IPN;
    unsigned short* const imgD = imgV + IVN;
    if (INA_NTN_TR && g == (int)blockIdx.x)   // once: rows / columns a shape never writes must read as zero
      for (int i = lane; i < (IPN + 2 * IVN) / 2; i += 64) reinterpret_cast<uint32_t*>(imgP)[i] = 0u;
    const int nw = E - g * NTN_WAVES < NTN_WAVES ? E - g * NTN_WAVES : NTN_WAVES;   // active waves of the group
    auto flush_dw = [&](int pp) {
      if (PAPER) return;
      if ((int)threadIdx.x < 2 * N * N) {
        const int sl = (int)threadIdx.x / (N * N), rem = (int)threadIdx.x - sl * N * N, sv = 2 * pp + sl;
        if (sv < h) {
          const float* src = dwl + ((pp & 1) * NTN_WAVES * 2 + sl) * NN1 + rem;
          float acc = 0.f;
          for (int w = 0; w < nw; ++w) acc += src[w * 2 * NN1];
          dw_slab[((long)g * h + sv) * N * N + rem] = acc;
        }
      }
    };
    __syncthreads();
    ntn_stage<MTH, NSW, true>(ntn_lds, p0, mpack, m2pack, wtpack, 2);
    stage_wait();
    __syncthreads();
    for (int p = p0; p < p1; ++p) {
      if (p > p0) flush_dw(p - 1);   // the previous pair's dw slots are complete (barrier at its end)
      const u16x8_t* buf = ntn_lds + ((p - p0) & 1) * FR * 64;
      if (p + 1 < p1) ntn_stage<MTH, NSW, true>(ntn_lds + ((p + 1 - p0) & 1) * FR * 64, p + 1, mpack, m2pack, wtpack, 2);
#if INA_NTN_TR
      if (act) {
        f32x4_t dTs[2][QT];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const int s = 2 * p + sl;
          const bool sok = s < h;   // (a padding slice runs on zero packs and stores into the trash tails)
          f32x4_t PT[2 * NKB];
#pragma unroll
          for (int mb = 0; mb < 2 * NKB; ++mb) {
            PT[mb] = Z4;
            if (mb < MTH) {
#pragma unroll
              for (int ka = 0; ka < NKA; ++ka) PT[mb] = mfma_bf16(buf[((sl * MTH + mb) * NKA + ka) * 64 + lane], Cf[ka], PT[mb]);
            }
          }
          u16x8_t PTf[NKB];
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) PTf[kb] = pack2(PT[2 * kb], PT[2 * kb + 1]);
          // P^T [b][c = n] -> I_P row (slice sl, class n) in the pair-fragment k order 8 (c >> 2) + 4 sl + (c & 3)
          {
            unsigned short* row = imgP + (8 * (n >> 2) + 4 * sl + (n & 3)) * PS + 4 * q;
#pragma unroll
            for (int mb = 0; mb < MTH; ++mb) {
              const u16x8_t& f = PTf[mb >> 1];
              const int o = 4 * (mb & 1);
              *reinterpret_cast<u16x4_t*>(row + 16 * mb) = u16x4_t{f[o], f[o + 1], f[o + 2], f[o + 3]};
            }
          }
          u16x8_t wt = {0, 0, 0, 0, 0, 0, 0, 0};
          float ws = 0.f;
          if (PAPER) ws = wvec[s];
          else wt = buf[(F1 + F2 + sl) * 64 + lane];
          float dwp = 0.f;
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            f32x4_t T = Z4;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) T = mfma_bf16(PTf[kb], Qf[qt][kb], T);   // rows c, cols query
            f32x4_t dV;
            if (PAPER) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                dV[r] = ws * dzC[qt][r];
                dwp += fmaxf(T[r], 0.f) * dzC[qt][r];
              }
            } else {
              dV = mfma_bf16(wt, dzA[qt], Z4);   // rows c, cols query
            }
            f32x4_t V;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              dTs[sl][qt][r] = T[r] > 0.f ? dV[r] : 0.f;
              V[r] = fmaxf(T[r], 0.f);
            }
            // rows c = 4q + r, cols query 16 qt + n -> I_V / I_dT row = query, cols c
            const int ro = (16 * qt + n) * VS + 4 * q;
            if (!PAPER)
              *reinterpret_cast<u16x4_t*>(imgV + ro) = u16x4_t{f2bf(V[0]), f2bf(V[1]), f2bf(V[2]), f2bf(V[3])};
            *reinterpret_cast<u16x4_t*>(imgD + ro) =
                u16x4_t{f2bf(dTs[sl][qt][0]), f2bf(dTs[sl][qt][1]), f2bf(dTs[sl][qt][2]), f2bf(dTs[sl][qt][3])};
          }
          lds_order();
          if (PAPER) {
            dwp = wave_sum(dwp);
            if (lane == 0 && sok) dw_slab[(long)ep * h + s] = dwp;
          } else {
            f32x4_t dw = Z4;   // dw[c][c'] = sum_q relu(T)[c][q] dz[q][c']
#pragma unroll
            for (int kq = 0; kq < KQ; ++kq) dw = mfma_bf16(tr_read8(imgV + kq * 32 * VS, VS, 0, q, n), dzB[kq], dw);
            float* const dst = dwl + (((p & 1) * NTN_WAVES + wave) * 2 + sl) * NN1;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(4 * q + r < N && n < N) ? (4 * q + r) * N + n : N * N] = dw[r];
          }
          // dP^T[b, c] = sum_q Q[q, b] dT[c, q]  (B = dT^T from I_dT)
          u16x8_t dTB[KQ];
#pragma unroll
          for (int kq = 0; kq < KQ; ++kq) dTB[kq] = tr_read8(imgD + kq * 32 * VS, VS, 0, q, n);
          lds_order();   // the next slice's image stores come after these reads
          f32x4_t dPT[2 * NKB];
#pragma unroll
          for (int mb = 0; mb < 2 * NKB; ++mb) {
            dPT[mb] = Z4;
            if (mb < MTH) {
#pragma unroll
              for (int kq = 0; kq < KQ; ++kq) dPT[mb] = mfma_bf16(QTf[mb][kq], dTB[kq], dPT[mb]);
            }
          }
          // dC^T[a, c] += sum_b M[a, b, s] dP[c, b]
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) {
            const u16x8_t dPf = pack2(dPT[2 * kb], dPT[2 * kb + 1]);
#pragma unroll
            for (int ma = 0; ma < MTH; ++ma)
              dCT[ma] = mfma_bf16(buf[(F1 + (sl * MTH + ma) * NKB + kb) * 64 + lane], dPf, dCT[ma]);
          }
          // dP -> bf16 [E*N][h*H] for the dM reduction GEMM
          unsigned short* const dpt = dp_out + (long)E * N * hH;
#pragma unroll
          for (int mb = 0; mb < MTH; ++mb)
            *reinterpret_cast<u16x4_t*>(sok ? dpb[mb] + s * H : dpt) =
                u16x4_t{f2bf(dPT[mb][0]), f2bf(dPT[mb][1]), f2bf(dPT[mb][2]), f2bf(dPT[mb][3])};
        }
        // dQ^T[b, q] += sum_{s in pair, c} P_s[c, b] dT_s[c, q]  (A = the pair's P from I_P)
        lds_order();
#pragma unroll
        for (int nb = 0; nb < MTH; ++nb) {
          const u16x8_t Pf = tr_read8(imgP, PS, 16 * nb, q, n);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) dQT[nb][qt] = mfma_bf16(Pf, pack2(dTs[0][qt], dTs[1][qt]), dQT[nb][qt]);
        }
        lds_order();
      }
#else
      if (act) {
        f32x4_t Ps[2][MTH], dTs[2][QT];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const int s = 2 * p + sl;
#pragma unroll
          for (int m = 0; m < MTH; ++m) Ps[sl][m] = Z4;
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) dTs[sl][qt] = Z4;
          // a padding slice (odd h, s = h) runs on the zero-padded packs -- all its values are zero -- and
          // stores into the trash tails: no branch between the pair's two slice chains, so the scheduler
          // can interleave them
          const bool sok = s < h;
          // P^T (rows b, cols c) and P (rows c, cols b) from the same fragments (operand swap)
          f32x4_t PT[2 * NKB];
#pragma unroll
          for (int mb = 0; mb < 2 * NKB; ++mb) {
            PT[mb] = Z4;
            if (mb < MTH) {
#pragma unroll
              for (int ka = 0; ka < NKA; ++ka) {
                const u16x8_t mf = buf[((sl * MTH + mb) * NKA + ka) * 64 + lane];
                PT[mb] = mfma_bf16(mf, Cf[ka], PT[mb]);
                Ps[sl][mb] = mfma_bf16(Cf[ka], mf, Ps[sl][mb]);
              }
            }
          }
          u16x8_t PTf[NKB];
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) PTf[kb] = pack2(PT[2 * kb], PT[2 * kb + 1]);
          u16x8_t wt = {0, 0, 0, 0, 0, 0, 0, 0};
          float ws = 0.f;
          if (PAPER) {
            ws = wvec[s];
          } else {
            wt = buf[(F1 + F2 + sl) * 64 + lane];
          }
          f32x4_t VT[2 * KQ], dTT[2 * KQ];
#pragma unroll
          for (int i = 0; i < 2 * KQ; ++i) VT[i] = dTT[i] = Z4;
          float dwp = 0.f;
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) {
            f32x4_t T = Z4, TT = Z4;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb) {
              T = mfma_bf16(PTf[kb], Qf[qt][kb], T);    // rows c, cols query
              TT = mfma_bf16(Qf[qt][kb], PTf[kb], TT);  // rows query, cols c
            }
            f32x4_t dV, dVT;
            if (PAPER) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                dV[r] = ws * dzC[qt][r];
                dVT[r] = ws * dzR[qt][r];
                dwp += fmaxf(TT[r], 0.f) * dzR[qt][r];
              }
            } else {
              dV = mfma_bf16(wt, dzA[qt], Z4);   // rows c, cols query
              dVT = mfma_bf16(dzA[qt], wt, Z4);  // rows query, cols c
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              dTs[sl][qt][r] = T[r] > 0.f ? dV[r] : 0.f;
              dTT[qt][r] = TT[r] > 0.f ? dVT[r] : 0.f;
            }
            VT[qt] = relu4(TT);
          }
          // per-episode dw contribution
          if (PAPER) {
            dwp = wave_sum(dwp);
            if (lane == 0 && sok) dw_slab[(long)ep * h + s] = dwp;
          } else {
            f32x4_t dw = Z4;
#pragma unroll
            for (int kq = 0; kq < KQ; ++kq) dw = mfma_bf16(pack2(VT[2 * kq], VT[2 * kq + 1]), dzB[kq], dw);
            float* const dst = dwl + (((p & 1) * NTN_WAVES + wave) * 2 + sl) * NN1;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(4 * q + r < N && n < N) ? (4 * q + r) * N + n : N * N] = dw[r];
          }
          // dP^T[b, c] = sum_q Q[q, b] dT[c, q]
          f32x4_t dPT[2 * NKB];
#pragma unroll
          for (int mb = 0; mb < 2 * NKB; ++mb) {
            dPT[mb] = Z4;
            if (mb < MTH) {
#pragma unroll
              for (int kq = 0; kq < KQ; ++kq)
                dPT[mb] = mfma_bf16(QTf[mb][kq], pack2(dTT[2 * kq], dTT[2 * kq + 1]), dPT[mb]);
            }
          }
          // dC^T[a, c] += sum_b M[a, b, s] dP[c, b]
#pragma unroll
          for (int kb = 0; kb < NKB; ++kb) {
            const u16x8_t dPf = pack2(dPT[2 * kb], dPT[2 * kb + 1]);
#pragma unroll
            for (int ma = 0; ma < MTH; ++ma)
              dCT[ma] = mfma_bf16(buf[(F1 + (sl * MTH + ma) * NKB + kb) * 64 + lane], dPf, dCT[ma]);
          }
          // dP -> bf16 [E*N][h*H] for the dM reduction GEMM
          unsigned short* const dpt = dp_out + (long)E * N * hH;
#pragma unroll
          for (int mb = 0; mb < MTH; ++mb)
            *reinterpret_cast<u16x4_t*>(sok ? dpb[mb] + s * H : dpt) =
                u16x4_t{f2bf(dPT[mb][0]), f2bf(dPT[mb][1]), f2bf(dPT[mb][2]), f2bf(dPT[mb][3])};
        }
        // dQ^T[b, q] += sum_{s in pair, c} P_s[c, b] dT_s[c, q]
#pragma unroll
        for (int nb = 0; nb < MTH; ++nb) {
          const u16x8_t Pf = pack2(Ps[0][nb], Ps[1][nb]);
#pragma unroll
          for (int qt = 0; qt < QT; ++qt) dQT[nb][qt] = mfma_bf16(Pf, pack2(dTs[0][qt], dTs[1][qt]), dQT[nb][qt]);
        }
      }
#endif
      stage_wait();
      __syncthreads();
    }
    if (p1 > p0) flush_dw(p1 - 1);   // read before the next group's first barrier pair
    if (act) {
      const bool split = gridDim.y > 1;
      float* dc_out = split ? pc + (long)blockIdx.y * E * N * H : dcls;
#pragma unroll
      for (int ma = 0; ma < MTH; ++ma) {
        const int a0 = 16 * ma + 4 * q;
        if (n < N && a0 < H) *reinterpret_cast<f32x4_t*>(dc_out + ((long)ep * N + n) * H + a0) = dCT[ma];
      }
      // query-row gradients: straight into de, or this split's compact [E][NQ][H] partial
      float* dq_base = split ? pq + ((long)blockIdx.y * E + ep) * NQ * H : de + rq0 * H;
#pragma unroll
      for (int nb = 0; nb < MTH; ++nb)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const int b0 = 16 * nb + 4 * q, qi = 16 * qt + n;
          if (qi < NQ && b0 < H) *reinterpret_cast<f32x4_t*>(dq_base + (long)qi * H + b0) = dQT[nb][qt];
        }
    }
  }
}

// sums of the slice-split partials, in split order (deterministic)
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

// ------------------------------------------------------------------------------------------
namespace ina {

static int finish_grid(long n) {
  const long g = (n + 255) / 256;
  return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);
}

static size_t ntn_lds_bytes(int MTH, bool paper, bool bwd, int N = 0) {
  const int NKA = (MTH + 1) / 2;
  const int fr = bwd ? (4 * MTH * NKA + (paper ? 0 : 2)) : (2 * MTH * NKA + (paper ? 0 : 1));
  // + the reference-head backward's dw slots [2 parities][waves][2 slices][N*N + 1] fp32
  const size_t dwl = (bwd && !paper) ? (size_t)2 * NTN_WAVES * 2 * (N * N + 1) * 4 : 0;
  // + (TR) the wave-private transpose images, 16-byte aligned after the dw slots
  const int KQ = 2;   // upper bound over the instantiated QT (<= 4)
  const size_t img = (bwd && INA_NTN_TR) ? 16 + (size_t)NTN_WAVES * (32 * (16 * MTH + 4) + 2 * 32 * KQ * 20) * 2 : 0;
  return (size_t)2 * fr * 64 * 16 + dwl + img;
}

int ntn_groups(int E) { return (E + NTN_WAVES - 1) / NTN_WAVES; }

template <int MTH, int QT, bool P>
static int ntn_fwd_t(const NtnArgs& a, hipStream_t st) {
  const int groups = (a.E + NTN_WAVES - 1) / NTN_WAVES;
  const int blocks = groups < a.blocks ? groups : a.blocks;
  const int ny = a.split > 1 ? a.split : 1;
  hipLaunchKernelGGL((ntn_fwd_kernel<MTH, QT, P>), dim3(blocks, ny), dim3(NTN_THREADS), ntn_lds_bytes(MTH, P, false),
                     st, a.cls, a.e, a.E, a.N, a.K, a.Q, a.H, a.h, (const u16x8_t*)a.mpack, (const u16x8_t*)a.wpack,
                     a.wvec, a.bias, a.probs, a.part);
  if (ny > 1) {
    const long n = (long)a.E * a.N * a.Q * a.N;
    hipLaunchKernelGGL(ntn_fwd_finish_kernel, dim3(finish_grid(n)), dim3(256), 0, st, a.part, ny, n, a.N, a.paper,
                       a.bias, a.probs);
  }
  INA_CHECK_LAUNCH();
  return 0;
}
template <int MTH, int QT, bool P>
static int ntn_bwd_t(const NtnArgs& a, hipStream_t st) {
  const int groups = (a.E + NTN_WAVES - 1) / NTN_WAVES;
  const int blocks = groups < a.blocks ? groups : a.blocks;
  const int ny = a.split > 1 ? a.split : 1;
  const size_t lds = ntn_lds_bytes(MTH, P, true, a.N);
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)ntn_bwd_kernel<MTH, QT, P>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return -1;
  hipLaunchKernelGGL((ntn_bwd_kernel<MTH, QT, P>), dim3(blocks, ny), dim3(NTN_THREADS), lds,
                     st, a.cls, a.e, a.E, a.N, a.K, a.Q, a.H, a.h, (const u16x8_t*)a.mpack, (const u16x8_t*)a.m2pack,
                     (const u16x8_t*)a.wtpack, a.wvec, a.dz, a.dcls, a.de, (unsigned short*)a.dp_out, a.dw_slab,
                     a.gscale, (unsigned short*)a.cls_bf, a.part, a.part2);
  if (ny > 1) {
    const long n = (long)a.E * a.N * a.H * (1 + a.Q);
    hipLaunchKernelGGL(ntn_bwd_finish_kernel, dim3(finish_grid(n)), dim3(256), 0, st, a.part, a.part2, ny, a.E, a.N,
                       a.K, a.Q, a.H, a.dcls, a.de);
  }
  INA_CHECK_LAUNCH();
  return 0;
}

#define INA_NTN_QT(FN, MTH, P)                       \
  if (QT == 1) return FN<MTH, 1, P>(a, st);          \
  if (QT == 2) return FN<MTH, 2, P>(a, st);          \
  if (QT == 4) return FN<MTH, 4, P>(a, st);
#define INA_NTN_DISPATCH(FN)                                              \
  const int QT = qt_needed <= 1 ? 1 : (qt_needed <= 2 ? 2 : (qt_needed <= 4 ? 4 : 0)); \
  if (QT == 0) return -1;                                                 \
  if (a.paper) {                                                          \
    if (MTH == 1) { INA_NTN_QT(FN, 1, true) }                             \
    if (MTH == 3) { INA_NTN_QT(FN, 3, true) }                             \
    if (MTH == 4) { INA_NTN_QT(FN, 4, true) }                             \
  } else {                                                                \
    if (MTH == 1) { INA_NTN_QT(FN, 1, false) }                            \
    if (MTH == 3) { INA_NTN_QT(FN, 3, false) }                            \
    if (MTH == 4) { INA_NTN_QT(FN, 4, false) }                            \
  }                                                                       \
  return -1;

// slice-split factor for small episode batches: fill ~256 workgroups, >= 2 slice pairs per split
int ntn_split(int E, int h) {
  const int groups = (E + NTN_WAVES - 1) / NTN_WAVES, npair = (h + 1) / 2;
  if (groups >= 64) return 1;
  int ny = 256 / groups;
  if (ny > npair / 2) ny = npair / 2;
  return ny > 1 ? ny : 1;
}

int ntn_fwd(const NtnArgs& a, hipStream_t st) {
  const int MTH = (a.H + 15) / 16, qt_needed = (a.N * a.Q + 15) / 16;
  if (a.N > 16) return -1;
  INA_NTN_DISPATCH(ntn_fwd_t)
}
int ntn_bwd(const NtnArgs& a, hipStream_t st) {
  const int MTH = (a.H + 15) / 16, qt_needed = (a.N * a.Q + 15) / 16;
  if (a.N > 16) return -1;
  INA_NTN_DISPATCH(ntn_bwd_t)
}

}  // namespace ina
