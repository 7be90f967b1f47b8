// Wide BiLSTM cell kernels (K2 for large hidden sizes, e.g. the paper configuration u=128, E=300,
// SURVEY 2.3 "paper config"; reference semantics model/graph.py:34-49 as in lstm.hip).
//
// The fused lane-ownership kernel (lstm.hip) keeps the whole recurrence in registers and is
// instantiated for u <= 32.  For wide layers the recurrence is split the cuDNN way: the input
// projection of every time step is ONE hipBLASLt GEMM (X W_x + b over all S*L tokens, both
// directions), each step's recurrent product h_{t-1} W_h is a batched GEMM over the two directions,
// and these kernels fuse everything elementwise around them:
//   fwd step: gates = Gx[t] + Gh; i,j,f,o activations; c' = c*sig(f+1) + sig(i)*tanh(j);
//             h' = tanh(c')*sig(o); stores h (bf16, recurrent operand), c (fp32), the activations
//             (bf16, for the backward) and the DropoutWrapper output in natural layout [S, L, 2u].
//   bwd step: dh = dH_out[t]*mask/kp + dh_rec; dc = dc_rec + dh*o*(1-tanh(c)^2); dG (pre-activation
//             gate gradients, bf16, written for the weight-gradient GEMMs); dc_rec' = dc*f.
// Gx is kept in fp32 (the fused kernel accumulates x W_x and h W_h in one fp32 MFMA chain).
// Layouts: direction-major [2][S][...]; direction 1 runs over reversed time (t = L-1-tau).
#include "ina_common.h"
#include "ina_launch.h"

using namespace ina;

namespace {

// one thread per (dir, s, unit); gates in TF order i, j, f, o at columns g*U + unit
__global__ __launch_bounds__(256) void lstm_wide_fwd_step_kernel(
    const float* __restrict__ gx,            // [2][S][L][4U] fp32: x W_x + b
    const float* __restrict__ gh,            // [2][S][4U] fp32: h_{t-1} W_h
    float* __restrict__ c,                   // [2][S][U] fp32 in/out
    unsigned short* __restrict__ hcur,       // [2][S][U] bf16 out (next step's GEMM operand)
    unsigned short* __restrict__ hall,       // [2][S][L][U] bf16 out (raw h, for dW_h)
    float* __restrict__ call,                // [2][S][L][U] fp32 out (cell states) or null
    unsigned short* __restrict__ acts,       // [2][S][L][4U] bf16 out (i, j, f, o activations) or null
    unsigned short* __restrict__ hout,       // [S][L][2U] bf16 (dropout applied)
    int S, int L, int U, int tau, uint32_t salt0, uint32_t salt1, uint32_t thr, float inv_kp, int drop) {
  const long total = 2L * S * U;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int dir = (int)(i / ((long)S * U));
    const long r = i - (long)dir * S * U;
    const int s = (int)(r / U), u = (int)(r - (long)s * U);
    const int t = dir ? (L - 1 - tau) : tau;
    const size_t gxo = (((size_t)dir * S + s) * L + t) * 4 * U;
    const size_t gho = ((size_t)dir * S + s) * 4 * U;
    const float zi = gx[gxo + u] + gh[gho + u];
    const float zj = gx[gxo + U + u] + gh[gho + U + u];
    const float zf = gx[gxo + 2 * U + u] + gh[gho + 2 * U + u];
    const float zo = gx[gxo + 3 * U + u] + gh[gho + 3 * U + u];
    const float ig = sigmoidf_(zi), jg = tanhf_(zj), fg = sigmoidf_(zf + 1.0f), og = sigmoidf_(zo);
    const float cn = c[i] * fg + ig * jg;
    const float hv = round_bf(tanhf_(cn) * og);
    c[i] = cn;
    hcur[i] = f2bf(hv);
    const size_t so = (((size_t)dir * S + s) * L + t) * U + u;
    hall[so] = f2bf(hv);
    if (call) call[so] = cn;
    if (acts) {
      acts[gxo + u] = f2bf(ig);
      acts[gxo + U + u] = f2bf(jg);
      acts[gxo + 2 * U + u] = f2bf(fg);
      acts[gxo + 3 * U + u] = f2bf(og);
    }
    float ho = hv;
    if (drop) {
      const uint32_t idx = ((uint32_t)s * L + t) * U + u;   // same index as the fused kernel / oracle
      ho = lstm_keep(dir ? salt1 : salt0, idx, thr) ? hv * inv_kp : 0.f;
    }
    hout[((size_t)s * L + t) * 2 * U + dir * U + u] = f2bf(ho);
  }
}

__global__ __launch_bounds__(256) void lstm_wide_bwd_step_kernel(
    const unsigned short* __restrict__ dH,   // [S][L][2U] bf16: gradient wrt the dropout output
    const float* __restrict__ dhrec,         // [2][S][U] fp32: dG_{t+1} W_h^T (zeros at the first step)
    float* __restrict__ dcrec,               // [2][S][U] fp32 in/out
    const float* __restrict__ call,          // [2][S][L][U] fp32 cell states
    const unsigned short* __restrict__ acts, // [2][S][L][4U] bf16
    unsigned short* __restrict__ dG,         // [2][S][L][4U] bf16 out (pre-activation gate grads)
    unsigned short* __restrict__ dGcur,      // [2][S][4U] bf16 out (this step, operand of dG W_h^T) or null
    int S, int L, int U, int tau, uint32_t salt0, uint32_t salt1, uint32_t thr, float inv_kp, int drop) {
  const long total = 2L * S * U;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int dir = (int)(i / ((long)S * U));
    const long r = i - (long)dir * S * U;
    const int s = (int)(r / U), u = (int)(r - (long)s * U);
    const int t = dir ? (L - 1 - tau) : tau;        // tau counts processing steps forward in time
    float dout = bf2f(dH[((size_t)s * L + t) * 2 * U + dir * U + u]);
    if (drop) {
      const uint32_t idx = ((uint32_t)s * L + t) * U + u;
      dout = lstm_keep(dir ? salt1 : salt0, idx, thr) ? dout * inv_kp : 0.f;
    }
    const size_t so = (((size_t)dir * S + s) * L + t) * U + u;
    const size_t go = (((size_t)dir * S + s) * L + t) * 4 * U;
    const float ig = bf2f(acts[go + u]), jg = bf2f(acts[go + U + u]), fg = bf2f(acts[go + 2 * U + u]),
                og = bf2f(acts[go + 3 * U + u]);
    const float cn = call[so];
    const float cp = tau > 0 ? call[so + (dir ? U : -(long)U)] : 0.f;   // c_{t-1} in processing order
    const float tc = tanhf_(cn);
    const float dh = dout + dhrec[i];
    const float dc = dcrec[i] + dh * og * (1.f - tc * tc);
    const float di = dc * jg * ig * (1.f - ig);
    const float dj = dc * ig * (1.f - jg * jg);
    const float df = dc * cp * fg * (1.f - fg);
    const float d_o = dh * tc * og * (1.f - og);
    dcrec[i] = dc * fg;
    const unsigned short bi = f2bf(di), bj = f2bf(dj), bff = f2bf(df), bo = f2bf(d_o);
    dG[go + u] = bi;
    dG[go + U + u] = bj;
    dG[go + 2 * U + u] = bff;
    dG[go + 3 * U + u] = bo;
    if (dGcur) {   // (the caller may read this step's rows of dG through a strided view instead)
      const size_t gc = ((size_t)dir * S + s) * 4 * U;
      dGcur[gc + u] = bi;
      dGcur[gc + U + u] = bj;
      dGcur[gc + 2 * U + u] = bff;
      dGcur[gc + 3 * U + u] = bo;
    }
  }
}

}  // namespace

namespace ina {

static int wide_grid(long total) {
  long g = (total + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

int lstm_wide_fwd_step(const LstmWideArgs& a, int tau, hipStream_t st) {
  hipLaunchKernelGGL(lstm_wide_fwd_step_kernel, dim3(wide_grid(2L * a.S * a.U)), dim3(256), 0, st,
                     (const float*)a.gx, a.gh, a.c, (unsigned short*)a.hcur, (unsigned short*)a.hall, a.call,
                     (unsigned short*)a.acts, (unsigned short*)a.hout, a.S, a.L, a.U, tau, a.salt0, a.salt1, a.thr,
                     a.inv_kp, a.drop);
  INA_CHECK_LAUNCH();
  return 0;
}

int lstm_wide_bwd_step(const LstmWideArgs& a, int tau, hipStream_t st) {
  hipLaunchKernelGGL(lstm_wide_bwd_step_kernel, dim3(wide_grid(2L * a.S * a.U)), dim3(256), 0, st,
                     (const unsigned short*)a.dH, a.dhrec, a.dcrec, a.call, (const unsigned short*)a.acts,
                     (unsigned short*)a.dG, (unsigned short*)a.dGcur, a.S, a.L, a.U, tau, a.salt0, a.salt1, a.thr,
                     a.inv_kp, a.drop);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina

// ==========================================================================================
// Persistent wide BiLSTM: the whole recurrence of a 32-sequence tile and one direction in ONE
// workgroup (NW = UP / 16 waves, 16 units per wave), U in {64, 100, 128} (the reference Base default
// u=100, the paper's u=128).  The per-step kernels above round-trip the recurrent GEMM's fp32 output
// (131 MB per step at the paper configuration) and relaunch 2 x L times; here
//   * each wave keeps ITS slice of W_h as MFMA A fragments in VGPRs for the whole sequence
//     (forward: 4 M-tiles x UP/32 K-steps; backward: UP*4/32 K-steps over the permuted gate columns);
//   * gates are computed transposed, G^T[gate rows, seqs] = W_h^T h^T (+ the precomputed x W_x + b),
//     with the row order chosen so lane group q holds, in M-tile m, the 4 gates of unit 16w + 4q + m:
//     a lane owns 4 CONTIGUOUS units (one 32-byte gate load / dG store, one 8-byte h write per tile);
//     c and h never leave the lane (the lane-ownership layout of lstm.hip);
//   * h_t is exchanged through a double-buffered LDS image [32 seqs][UP] bf16 (the next step's B
//     operand), ONE workgroup barrier per step; the same image feeds coalesced row copies of the
//     attention input (DropoutWrapper applied) and the backward's h_{t-1} stash;
//   * every global input of a step (forward: x W_x; backward: activations, cells, attention gradient)
//     is loaded one step ahead into ping-pong registers (loops unrolled by two), so HBM latency hides
//     behind the previous step's recurrence instead of sitting on the serial chain;
//   * the activation / cell stash is tile-major (WideStash): 512 contiguous bytes per wave access;
//   * backward: dG (bf16) goes to an LDS image [32][4 UP] and is contracted with the backward W_h
//     fragments, whose rows land dh of unit 16w + 4q + r in accumulator register r of lane group q --
//     the lane that owns that unit's gates;
//   * backward, optional (dxp): the input gradient's position columns dX_pos = dG W_pos^T (<= 16 columns)
//     from the same LDS image -- wave w contracts 16-sequence tile w & 1 over 128 of the gate columns
//     (4 MFMAs per step), the UP / 32 partials per tile are summed in a fixed order through LDS one step
//     later.  This replaces a separate GEMM pass over the whole 2.4 GB dG at the paper configuration.
// Gate columns are permuted to c = 4u + g (unit-major, the 4 gates of a unit adjacent).
// ops/packing.py::pack_lstm_wide builds the fragments and is checked by tests/test_packing.py's
// MFMA-layout emulation.
// ==========================================================================================
namespace {

template <int U>
struct WideCfg {
  static_assert(U % 4 == 0, "a lane owns 4 contiguous units: U must be a multiple of 4");
  static constexpr int UP = (U + 31) / 32 * 32;
  static constexpr int NW = UP / 16;     // waves per workgroup
  static constexpr int M = 4;            // forward M-tiles per wave (16 gate rows = 4 units)
  static constexpr int KS = UP / 32;     // forward K-steps (input units)
  static constexpr int G4 = 4 * UP;      // permuted gate columns
  static constexpr int KS2 = G4 / 32;    // backward K-steps (gate columns)
  static constexpr int NT = 2;           // 16-sequence tiles per workgroup
  // LDS image row strides: +32 bytes, i.e. consecutive rows 2 bank slots (of 16 B) apart.  The MFMA B
  // operand reads (ds_read_b128: 16 rows n x chunk 4 ks + q per lane group {0-3,12-15 | q} u {4-11 | q+1})
  // then land rows of one q parity on even and the other on odd slots, pairwise distinct: conflict-free.
  // (+16 bytes put lane 12 and lane 27 on one slot: a 2-way conflict in every lane group, 44-46% of the
  // LDS cycles at the paper configuration, verdict r3 #5; an XOR swizzle costs per-lane addresses and
  // spilled the backward.)
  static constexpr int HS = UP + 16;     // h image row stride (elements)
  static constexpr int GS = G4 + 16;     // dG image row stride
  static constexpr int SEQ = NT * 16;
};

INA_DEVICE uint32_t pack_bf2(float a, float b) {
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  const bf2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

}  // namespace

INA_DEVICE uint32_t pack_h2(float a, float b) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, v);
}
INA_DEVICE float2 unpack_h2(uint32_t v) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t h = __builtin_bit_cast(h2_t, v);
  return float2{(float)h.x, (float)h.y};
}

// Tile-major stash (internal to the forward/backward pair, any layout works): per (dir, tile, t) one
// contiguous block, [NW][M][NT][64 lanes] x uint2 (4 bf16 activations) and [NW][NT][64] x uint2
// (the 4 fp16 cells of a lane's 4 units), so every stash load/store of a wave is 512 contiguous bytes.
template <int U>
struct WideStash {
  using C = WideCfg<U>;
  static constexpr int ASTEP = C::NW * C::M * C::NT * 64;   // uint2 per (dir, tile, t)
  static constexpr int CSTEP = C::NW * C::NT * 64;
};

template <int U>
__global__ __launch_bounds__(WideCfg<U>::NW * 64) void lstm_wide_seq_fwd_kernel(
    const unsigned short* __restrict__ gx, const float* __restrict__ bx, const u16x8_t* __restrict__ apk, int S, int L,
    unsigned short* __restrict__ hprev, uint2* __restrict__ acts, uint2* __restrict__ cst,
    unsigned short* __restrict__ hout, uint32_t salt0, uint32_t salt1, uint32_t thr, float inv_kp, int drop,
    int stash, int hld, long hdo) {
  using C = WideCfg<U>;
  using Z = WideStash<U>;
  constexpr int UP = C::UP, NW = C::NW, M = C::M, KS = C::KS, G4 = C::G4, NT = C::NT, HS = C::HS, SEQ = C::SEQ;
  constexpr int NTH = NW * 64;
  __shared__ __attribute__((aligned(16))) unsigned short himg[2][SEQ * HS];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, n = lane & 15;
  const int dir = blockIdx.y, s0 = blockIdx.x * SEQ;
  const uint32_t salt = dir ? salt1 : salt0, thr16 = thr >> 16;
  u16x8_t A[M][KS];
  {
    const u16x8_t* ap = apk + (size_t)(dir * NW + w) * M * KS * 64 + lane;
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) A[m][ks] = ap[(m * KS + ks) * 64];
  }
  for (int i = threadIdx.x; i < SEQ * HS; i += NTH) reinterpret_cast<uint32_t*>(himg)[i] = 0u;   // both images
  __syncthreads();
  float c[M][NT];
  int srow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int s = s0 + nt * 16 + n;
    srow[nt] = s < S ? s : S - 1;   // tail rows recompute the last sequence (their stash rows are padding)
#pragma unroll
    for (int m = 0; m < M; ++m) c[m][nt] = 0.f;
  }
  const int u0 = 16 * w + 4 * q;   // the lane's 4 contiguous units u0 + m (packing.py _wide_idx)
  float4 bias[M];                  // pre-scaled gate biases of the lane's units (forget gate +1)
#pragma unroll
  for (int m = 0; m < M; ++m) bias[m] = *reinterpret_cast<const float4*>(bx + dir * G4 + 4 * (u0 + m));
  uint2* const actp = acts + (size_t)(dir * gridDim.x + blockIdx.x) * L * Z::ASTEP + w * (M * NT * 64) + lane;
  uint2* const cstp = cst + (size_t)(dir * gridDim.x + blockIdx.x) * L * Z::CSTEP + w * (NT * 64) + lane;
  // x W_x of one step (bf16, 4 gates x 4 units = 32 contiguous bytes per lane and tile): software-
  // pipelined one step ahead so the HBM latency hides behind the previous step's recurrence
  auto load_gx = [&](int t, uint4 (&g)[NT][2]) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const uint4* src = reinterpret_cast<const uint4*>(gx + ((size_t)srow[nt] * L + t) * (2 * G4) + dir * G4 + 4 * u0);
      g[nt][0] = src[0];
      g[nt][1] = src[1];
    }
  };
  constexpr int CH = UP / 8, NCH = SEQ * CH;   // row copies: one 16-byte chunk (8 units) per thread and pass
  // one step; gcur holds its x W_x, gnx receives the next step's (ping-pong buffers: the loop below is
  // unrolled by two so no register copy forces an early wait on the prefetch)
  auto step = [&](int tau, const uint4 (&gcur)[NT][2], uint4 (&gnx)[NT][2]) __attribute__((always_inline)) {
    const int t = dir ? L - 1 - tau : tau;
    const int tn = tau + 1 < L ? (dir ? t - 1 : t + 1) : t;
    load_gx(tn, gnx);
    const unsigned short* hin = himg[tau & 1];
    unsigned short* hnx = himg[(tau + 1) & 1];
    if (stash) {   // this step's recurrent input h_{t-1} -> hprev row s L + t of direction dir (the dW_h GEMM's
                   // rows: row stride hld, direction offset hdo elements)
      for (int i = threadIdx.x; i < NCH; i += NTH) {
        const int r = i / CH, ch = i - r * CH, s = s0 + r;
        if (s < S)
          *reinterpret_cast<u16x8_t*>(hprev + dir * hdo + ((size_t)s * L + t) * hld + 8 * ch) =
              *reinterpret_cast<const u16x8_t*>(hin + r * HS + 8 * ch);
      }
    }
    u16x8_t B[NT][KS];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) B[nt][ks] = *reinterpret_cast<const u16x8_t*>(hin + (nt * 16 + n) * HS + 32 * ks + 8 * q);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const uint32_t gw[8] = {gcur[nt][0].x, gcur[nt][0].y, gcur[nt][0].z, gcur[nt][0].w,
                              gcur[nt][1].x, gcur[nt][1].y, gcur[nt][1].z, gcur[nt][1].w};
      float hv[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        f32x4_t acc = {bias[m].x + bf2f((unsigned short)gw[2 * m]), bias[m].y + bf2f((unsigned short)(gw[2 * m] >> 16)),
                       bias[m].z + bf2f((unsigned short)gw[2 * m + 1]),
                       bias[m].w + bf2f((unsigned short)(gw[2 * m + 1] >> 16))};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = mfma_bf16(A[m][ks], B[nt][ks], acc);
        const float ig = sigmoid_l2(acc[0]), jg = tanh_l2(acc[1]), fg = sigmoid_l2(acc[2]), og = sigmoid_l2(acc[3]);
        const float cn = c[m][nt] * fg + ig * jg;
        c[m][nt] = cn;
        hv[m] = tanh_l2(cn * (2.f * LOG2E_F)) * og;
        if (stash) actp[(size_t)t * Z::ASTEP + (m * NT + nt) * 64] = uint2{pack_bf2(ig, jg), pack_bf2(fg, og)};
      }
      *reinterpret_cast<uint2*>(hnx + (nt * 16 + n) * HS + u0) = uint2{pack_bf2(hv[0], hv[1]), pack_bf2(hv[2], hv[3])};
    }
    if (stash) {   // fp16 cells (|c| <= L: far inside range, 11-bit mantissa), the lane's 4 units per store
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        cstp[(size_t)t * Z::CSTEP + nt * 64] = uint2{pack_h2(c[0][nt], c[1][nt]), pack_h2(c[2][nt], c[3][nt])};
    }
    __syncthreads();   // hnx complete; every wave is past its reads of hin
    // attention input h_t (DropoutWrapper: keep ? h / keep_prob : 0, one hash per unit pair as the
    // fused kernels / oracle) -> hout[s][t][dir U + u], two units per 4-byte store
    for (int i = threadIdx.x; i < SEQ * (UP / 2); i += NTH) {
      const int r = i / (UP / 2), u = 2 * (i - r * (UP / 2)), s = s0 + r;
      if (s >= S || u >= U) continue;
      const uint32_t hv = *reinterpret_cast<const uint32_t*>(hnx + r * HS + u);
      uint32_t o = hv;
      if (drop) {
        const uint32_t x = dropout_mix(salt, (((uint32_t)s * L + t) * U + u) >> 1);
        const float a = bf2f((unsigned short)hv), b = bf2f((unsigned short)(hv >> 16));
        o = pack_bf2((x & 0xFFFFu) < thr16 ? a * inv_kp : 0.f, (x >> 16) < thr16 ? b * inv_kp : 0.f);
      }
      *reinterpret_cast<uint32_t*>(hout + ((size_t)s * L + t) * 2 * U + dir * U + u) = o;
    }
  };
  uint4 g0[NT][2], g1[NT][2];
  load_gx(dir ? L - 1 : 0, g0);
  int tau = 0;
  for (; tau + 1 < L; tau += 2) {
    step(tau, g0, g1);
    step(tau + 1, g1, g0);
  }
  if (tau < L) step(tau, g0, g1);
}

template <int U>
__global__ __launch_bounds__(WideCfg<U>::NW * 64) void lstm_wide_seq_bwd_kernel(
    const unsigned short* __restrict__ dH, const uint2* __restrict__ acts, const uint2* __restrict__ cst,
    const u16x8_t* __restrict__ a2pk, unsigned short* __restrict__ dG, int S, int L, uint32_t salt0, uint32_t salt1,
    uint32_t thr, float inv_kp, int drop, const u16x8_t* __restrict__ wpk, float* __restrict__ dxp, int np) {
  using C = WideCfg<U>;
  using Z = WideStash<U>;
  constexpr int UP = C::UP, NW = C::NW, M = C::M, G4 = C::G4, KS2 = C::KS2, NT = C::NT, GS = C::GS, SEQ = C::SEQ;
  constexpr int NTH = NW * 64, NG = NW / 2;   // NG dX_pos partials per 16-sequence tile (4 K-steps each)
  static_assert(NW % 2 == 0 && 4 * NG == KS2, "dX_pos: NW / 2 wave pairs x 4 K-steps cover the gate columns");
  __shared__ __attribute__((aligned(16))) unsigned short gimg[2][SEQ * GS];
  __shared__ __attribute__((aligned(16))) float pimg[2][NG * NT * 16 * 16];   // [buf][kg][nt][seq][16 cols]
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane >> 4, n = lane & 15;
  const int dir = blockIdx.y, s0 = blockIdx.x * SEQ;
  const uint32_t salt = dir ? salt1 : salt0;
  u16x8_t A2[KS2];
  {
    const u16x8_t* ap = a2pk + (size_t)(dir * NW + w) * KS2 * 64 + lane;
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) A2[ks] = ap[ks * 64];
  }
  const int ntw = w & 1, kg = w >> 1;   // dX_pos: this wave's tile and K-step group
  u16x8_t Wp[4];                        // W_pos^T fragments (rows = position columns, zero rows >= np)
  if (dxp != nullptr) {
    const u16x8_t* wp = wpk + ((size_t)dir * KS2 + 4 * kg) * 64 + lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) Wp[k] = wp[k * 64];
  }
  // sum of the NG partials of one processed step (buffer buf, time t) -> dxp[dir][s*L + t][0 .. np)
  auto pos_reduce = [&](int buf, int t) {
    for (int i = threadIdx.x; i < SEQ * 16; i += NTH) {
      const int sl = i >> 4, j = i & 15, s = s0 + sl;
      if (s < S && j < np) {
        float v = 0.f;
#pragma unroll
        for (int g = 0; g < NG; ++g) v += pimg[buf][((g * NT + (sl >> 4)) * 16 + (sl & 15)) * 16 + j];
        dxp[(((size_t)dir * S + s) * L + t) * np + j] = v;
      }
    }
  };
  // a step's partial is stored one step later, just before that step's barrier: the store does not wait
  // on its MFMA chain, and the sum still runs right after that barrier
  f32x4_t pacc = {0.f, 0.f, 0.f, 0.f};
  auto pos_store = [&](int buf) {
    *reinterpret_cast<f32x4_t*>(&pimg[buf][((kg * NT + ntw) * 16 + n) * 16 + 4 * q]) = pacc;
  };
  int srow[NT];
  bool sval[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int s = s0 + nt * 16 + n;
    sval[nt] = s < S;
    srow[nt] = sval[nt] ? s : S - 1;
  }
  const int u0 = 16 * w + 4 * q;   // the lane's 4 contiguous units (the forward's ownership)
  const bool uval = u0 < U;        // U % 4 == 0: a lane's units are all real or all padding
  const uint2* const actp = acts + (size_t)(dir * gridDim.x + blockIdx.x) * L * Z::ASTEP + w * (M * NT * 64) + lane;
  const uint2* const cstp = cst + (size_t)(dir * gridDim.x + blockIdx.x) * L * Z::CSTEP + w * (NT * 64) + lane;
  // one step's inputs, loaded a step ahead: activations, the previous step's cells, attention gradient
  struct In {
    uint2 a[M][NT];
    uint2 cp[NT];
    uint2 dout[NT];   // raw attention gradient of the 4 units (bf16): no use of the loaded values here
  };
  auto load_in = [&](int tau, In& v) {
    const int t = dir ? L - 1 - tau : tau;
    const int tp = tau > 0 ? (dir ? t + 1 : t - 1) : t;   // the step before in processing order
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) v.a[m][nt] = actp[(size_t)t * Z::ASTEP + (m * NT + nt) * 64];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      v.cp[nt] = cstp[(size_t)tp * Z::CSTEP + nt * 64];
      if (tau == 0) v.cp[nt] = uint2{0u, 0u};
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)   // padding units: any valid address, masked at use
      v.dout[nt] = *reinterpret_cast<const uint2*>(dH + ((size_t)srow[nt] * L + t) * 2 * U + dir * U + min(u0, U - 4));
  };
  f32x4_t dhr[NT];     // dh of units u0 + r (register r), from the previous processed step
  float dcr[M][NT];
  uint2 cn2[NT];       // this step's cells (the previous iteration's c_{t-1})
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    dhr[nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    cn2[nt] = cstp[(size_t)(dir ? 0 : L - 1) * Z::CSTEP + nt * 64];
#pragma unroll
    for (int m = 0; m < M; ++m) dcr[m][nt] = 0.f;
  }
  auto step = [&](int tau, const In& cur, In& nx) __attribute__((always_inline)) {
    const int t = dir ? L - 1 - tau : tau;
    load_in(tau > 0 ? tau - 1 : 0, nx);
    unsigned short* gcur = gimg[tau & 1];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float2 c01 = unpack_h2(cn2[nt].x), c23 = unpack_h2(cn2[nt].y);
      const float2 p01 = unpack_h2(cur.cp[nt].x), p23 = unpack_h2(cur.cp[nt].y);
      const float cnv[M] = {c01.x, c01.y, c23.x, c23.y}, cpv[M] = {p01.x, p01.y, p23.x, p23.y};
      const size_t row = (size_t)srow[nt] * L + t;   // dG [S*L][2][G4]: both directions on one row
      const float dov[M] = {bf2f((unsigned short)cur.dout[nt].x), bf2f((unsigned short)(cur.dout[nt].x >> 16)),
                            bf2f((unsigned short)cur.dout[nt].y), bf2f((unsigned short)(cur.dout[nt].y >> 16))};
      uint32_t gw[2 * M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int u = u0 + m;
        const uint2 av = cur.a[m][nt];
        const float ig = bf2f((unsigned short)av.x), jg = bf2f((unsigned short)(av.x >> 16));
        const float fg = bf2f((unsigned short)av.y), og = bf2f((unsigned short)(av.y >> 16));
        const float tc = tanh_l2(cnv[m] * (2.f * LOG2E_F));
        float dout = 0.f;
        if (uval && sval[nt]) {   // DropoutWrapper on the attention gradient (same hash as the forward)
          dout = dov[m];
          if (drop) dout = lstm_keep(salt, ((uint32_t)srow[nt] * L + t) * U + u, thr) ? dout * inv_kp : 0.f;
        }
        const float dh = dout + dhr[nt][m];
        const float dc = dcr[m][nt] + dh * og * (1.f - tc * tc);
        dcr[m][nt] = dc * fg;
        gw[2 * m] = pack_bf2(dc * jg * (ig - ig * ig), dc * ig * (1.f - jg * jg));
        gw[2 * m + 1] = pack_bf2(dc * cpv[m] * (fg - fg * fg), dh * tc * (og - og * og));
      }
      const uint4 g_lo = {gw[0], gw[1], gw[2], gw[3]}, g_hi = {gw[4], gw[5], gw[6], gw[7]};
      if (sval[nt]) {
        uint4* dst = reinterpret_cast<uint4*>(dG + row * (2 * G4) + dir * G4 + 4 * u0);
        dst[0] = g_lo;
        dst[1] = g_hi;
      }
      uint4* li = reinterpret_cast<uint4*>(gcur + (nt * 16 + n) * GS + 4 * u0);
      li[0] = g_lo;
      li[1] = g_hi;
      cn2[nt] = cur.cp[nt];
    }
    if (dxp != nullptr && tau + 1 < L) pos_store((tau + 1) & 1);
    __syncthreads();   // the dG image of this step is complete (and the previous step's dX_pos partials)
    if (tau > 0) {     // dh_{t-1} = dG W_h^T: two accumulators per tile (shorter dependent MFMA chains)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS2; ks += 2) {
          a0 = mfma_bf16(A2[ks], *reinterpret_cast<const u16x8_t*>(gcur + (nt * 16 + n) * GS + 32 * ks + 8 * q), a0);
          a1 = mfma_bf16(A2[ks + 1], *reinterpret_cast<const u16x8_t*>(gcur + (nt * 16 + n) * GS + 32 * ks + 32 + 8 * q), a1);
        }
        dhr[nt] = a0 + a1;
      }
    }
    if (dxp != nullptr) {
      if (tau + 1 < L) pos_reduce((tau + 1) & 1, dir ? L - 2 - tau : tau + 1);
      const unsigned short* br = gcur + (ntw * 16 + n) * GS + 128 * kg + 8 * q;
      pacc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 4; ++k) pacc = mfma_bf16(Wp[k], *reinterpret_cast<const u16x8_t*>(br + 32 * k), pacc);
    }
  };
  In b0, b1;   // ping-pong prefetch buffers (loop unrolled by two)
  load_in(L - 1, b0);
  int tau = L - 1;
  for (; tau >= 1; tau -= 2) {
    step(tau, b0, b1);
    step(tau - 1, b1, b0);
  }
  if (tau == 0) step(0, b0, b1);
  if (dxp != nullptr) {
    pos_store(0);
    __syncthreads();   // the last processed step's (tau = 0) partials
    pos_reduce(0, dir ? L - 1 : 0);
  }
}

namespace ina {

bool lstm_wide_seq_supported(int U) { return U == 64 || U == 100 || U == 128; }

template <int U>
static int wide_seq_fwd_t(const WideSeqArgs& a, hipStream_t st) {
  using C = WideCfg<U>;
  const dim3 grid((a.S + C::SEQ - 1) / C::SEQ, 2);
  hipLaunchKernelGGL(lstm_wide_seq_fwd_kernel<U>, grid, dim3(C::NW * 64), 0, st, (const unsigned short*)a.gx, a.bx,
                     (const u16x8_t*)a.apk, a.S, a.L, (unsigned short*)a.hprev, (uint2*)a.acts,
                     (uint2*)a.cst, (unsigned short*)a.hout, a.salt0,
                     a.salt1, a.thr, a.inv_kp, a.drop, a.stash, a.hld, a.hdo);
  INA_CHECK_LAUNCH();
  return 0;
}
template <int U>
static int wide_seq_bwd_t(const WideSeqArgs& a, hipStream_t st) {
  using C = WideCfg<U>;
  const dim3 grid((a.S + C::SEQ - 1) / C::SEQ, 2);
  hipLaunchKernelGGL(lstm_wide_seq_bwd_kernel<U>, grid, dim3(C::NW * 64), 0, st, (const unsigned short*)a.dH,
                     (const uint2*)a.acts, (const uint2*)a.cst, (const u16x8_t*)a.a2pk, (unsigned short*)a.dG, a.S, a.L,
                     a.salt0, a.salt1, a.thr, a.inv_kp, a.drop, (const u16x8_t*)a.wpk, a.dxp, a.np);
  INA_CHECK_LAUNCH();
  return 0;
}

int lstm_wide_seq_fwd(const WideSeqArgs& a, hipStream_t st) {
  if (a.U == 64) return wide_seq_fwd_t<64>(a, st);
  if (a.U == 100) return wide_seq_fwd_t<100>(a, st);
  if (a.U == 128) return wide_seq_fwd_t<128>(a, st);
  return -1;
}
int lstm_wide_seq_bwd(const WideSeqArgs& a, hipStream_t st) {
  if (a.U == 64) return wide_seq_bwd_t<64>(a, st);
  if (a.U == 100) return wide_seq_bwd_t<100>(a, st);
  if (a.U == 128) return wide_seq_bwd_t<128>(a, st);
  return -1;
}

}  // namespace ina

// ------------------------------------------------------------------------------------------
// Wide encoder input (K1 at wide shapes): Xb[s*L + t] = bf16 [word row ; pos1 row ; pos2 row] of token
// (inst[s], t) -- one pass instead of a word gather (fp32), a cast, two position gathers and a concat.
// One wave per token row (grid-stride), two columns (one 4-byte store) per lane and pass.
// ------------------------------------------------------------------------------------------
// WB: the word table is a cached bf16 copy (frozen tables, ops/wide.py::word_table_bf16): half the
// bytes of the random row reads.  RW rows per wave, every row's index chain (inst -> word id) and word
// vector loads issued before the first store: one row per wave left the kernel latency-bound on that
// dependent chain (646 us at the paper configuration, ~2.5 TB/s).
template <bool WB, int RW>
__global__ __launch_bounds__(256) void wide_x_gather_kernel(const int* __restrict__ inst, int S, int L,
                                                            const int* __restrict__ word, const int* __restrict__ pos1,
                                                            const int* __restrict__ pos2, const void* __restrict__ wemb_v,
                                                            int E, const float* __restrict__ p1emb,
                                                            const float* __restrict__ p2emb, int PD, int DP,
                                                            unsigned short* __restrict__ xb, int ldx) {
  const int lane = threadIdx.x & 63;
  const int D = E + 2 * PD;
  const long rows = (long)S * L;
  const long r0 = ((long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * RW;
  if (r0 >= rows) return;
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  long tok[RW], wbase[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const long r = r0 + i < rows ? r0 + i : rows - 1;
    const int s = (int)(r / L), t = (int)(r - (long)s * L);
    tok[i] = (long)inst[s] * L + t;
  }
  int p1v[RW], p2v[RW];   // position ids of all RW rows loaded with the word ids (no per-row chains below)
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    wbase[i] = (long)word[tok[i]] * E;
    p1v[i] = pos1[tok[i]];
    p2v[i] = pos2[tok[i]];
  }
  int c0 = 0;
  if ((E & 3) == 0) {   // word columns, 4 per lane and pass: all RW rows' loads in flight together
    for (int c = 4 * lane; c < E; c += 256) {
      uint2 v[RW];
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        if constexpr (WB) {
          v[i] = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(wemb_v) + wbase[i] + c);
        } else {
          const float4 f = *reinterpret_cast<const float4*>(static_cast<const float*>(wemb_v) + wbase[i] + c);
          const bf2_t lo = {(__bf16)f.x, (__bf16)f.y}, hi = {(__bf16)f.z, (__bf16)f.w};
          v[i] = uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
        }
      }
#pragma unroll
      for (int i = 0; i < RW; ++i)
        if (r0 + i < rows) *reinterpret_cast<uint2*>(xb + (r0 + i) * ldx + c) = v[i];
    }
    c0 = E;
  }
  // position columns, the ones column (index D) and zero padding up to DP (and the word columns when E % 4)
  if (DP - c0 <= 64) {   // one column per lane: the RW rows' table loads all in flight, then the stores
    const int c = c0 + lane;
    const int cp = c - E < PD ? c - E : c - E - PD;   // column inside its position table (c in [E, D))
    float vv[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      float wv = 0.f;
      if (c < E) {
        if constexpr (WB)
          wv = bf2f(static_cast<const unsigned short*>(wemb_v)[wbase[i] + c]);
        else
          wv = static_cast<const float*>(wemb_v)[wbase[i] + c];
      }
      const float pv = (c >= E && c < D) ? (c < E + PD ? p1emb : p2emb)[(long)(c < E + PD ? p1v[i] : p2v[i]) * PD + cp] : 0.f;
      vv[i] = c < E ? wv : c < D ? pv : c == D ? 1.f : 0.f;
    }
#pragma unroll
    for (int i = 0; i < RW; ++i)
      if (c < DP && r0 + i < rows) xb[(r0 + i) * ldx + c] = f2bf(vv[i]);
    return;
  }
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    if (r0 + i >= rows) break;
    const float* q1 = p1emb + (long)p1v[i] * PD;
    const float* q2 = p2emb + (long)p2v[i] * PD;
    unsigned short* dst = xb + (r0 + i) * ldx;
    for (int c = c0 + lane; c < DP; c += 64) {
      float wv = 0.f;
      if (c < E) {
        if constexpr (WB)
          wv = bf2f(static_cast<const unsigned short*>(wemb_v)[wbase[i] + c]);
        else
          wv = static_cast<const float*>(wemb_v)[wbase[i] + c];
      }
      const float v = c < E ? wv : c < E + PD ? q1[c - E] : c < D ? q2[c - E - PD] : c == D ? 1.f : 0.f;
      dst[c] = f2bf(v);
    }
  }
}

// Position-table gradients from the input gradient's position columns, for FewRel's shifted-arange
// ids (pos[i][t] = pos[i][0] + t, ops/sampler.py::positions_are_shifted): table tb row p collects
// dX[s][p - p0(s)][E + tb PD + c] over the sequences s with 0 <= p - p0(s) < L.  Thread = one output
// (tb, p, c), grid.y = sequence chunks -> partials [chunks][2][P2][PD] (summed in order by the caller:
// deterministic, no atomics).  dxp = dX's position columns, [planes][S*L][2PD] fp32 (planes = 2: the two
// directions' contributions as the fused BiLSTM backward writes them, summed here).
__global__ __launch_bounds__(256) void wide_pos_grad_kernel(const float* __restrict__ dxp, const int* __restrict__ inst,
                                                            const int* __restrict__ pos1, const int* __restrict__ pos2,
                                                            int S, int L, int PD, int P2, int chunk, int planes,
                                                            float* __restrict__ part) {
  // The per-sequence first positions p0(s) of both tables are staged through LDS a tile at a time by the
  // whole block (the inst[s] -> pos[] load chain is paid once per tile, in parallel, instead of serially
  // by every thread on every sequence).
  constexpr int TILE = 512;
  __shared__ int off[2][TILE];
  const int o = blockIdx.x * 256 + threadIdx.x;
  const int nout = 2 * P2 * PD;
  const bool live = o < nout;
  const int c = o % PD, p = (o / PD) % P2, tb = live ? o / (PD * P2) : 0;
  const int s0 = blockIdx.y * chunk, s1 = min(S, s0 + chunk);
  const long plane = (long)S * L * 2 * PD;
  float acc = 0.f;
  for (int b = s0; b < s1; b += TILE) {
    const int n = min(TILE, s1 - b);
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += 256) {
      const long r = (long)inst[b + j] * L;
      off[0][j] = pos1[r];
      off[1][j] = pos2[r];
    }
    __syncthreads();
    if (live)
      for (int j = 0; j < n; ++j) {
        const int t = p - off[tb][j];
        if (t >= 0 && t < L) {
          const long i = ((long)(b + j) * L + t) * 2 * PD + tb * PD + c;
          acc += planes == 2 ? dxp[i] + dxp[i + plane] : dxp[i];
        }
      }
  }
  if (live) part[(long)blockIdx.y * nout + o] = acc;
}

namespace ina {

int wide_x_gather(const int* inst, int S, int L, const int* word, const int* pos1, const int* pos2, const void* wemb,
                  bool wemb_bf16, int E, const float* p1emb, const float* p2emb, int PD, int DP, void* xb, int ldx,
                  hipStream_t st) {
#ifndef INA_WXG_RW
#define INA_WXG_RW 4   // rows per wave: 4 -> 383 us, 8 -> 415 us, 16 -> 477 us at the paper configuration (profiles/r5_rw)
#endif
  constexpr int RW = INA_WXG_RW;   // rows per wave
  const long rows = (long)S * L;
  const long blocks = (rows + 4 * RW - 1) / (4 * RW);
  if (blocks < 1) return 0;
  if (blocks >= (1L << 31)) return -1;
  if (wemb_bf16)
    hipLaunchKernelGGL((wide_x_gather_kernel<true, RW>), dim3((int)blocks), dim3(256), 0, st, inst, S, L, word, pos1,
                       pos2, wemb, E, p1emb, p2emb, PD, DP, (unsigned short*)xb, ldx);
  else
    hipLaunchKernelGGL((wide_x_gather_kernel<false, RW>), dim3((int)blocks), dim3(256), 0, st, inst, S, L, word, pos1,
                       pos2, wemb, E, p1emb, p2emb, PD, DP, (unsigned short*)xb, ldx);
  INA_CHECK_LAUNCH();
  return 0;
}

int wide_pos_grad(const float* dxp, const int* inst, const int* pos1, const int* pos2, int S, int L, int PD, int P2,
                  int chunks, int planes, float* part, hipStream_t st) {
  const int nout = 2 * P2 * PD;
  const int chunk = (S + chunks - 1) / chunks;
  hipLaunchKernelGGL(wide_pos_grad_kernel, dim3((nout + 255) / 256, chunks), dim3(256), 0, st, dxp, inst, pos1, pos2, S,
                     L, PD, P2, chunk, planes, part);
  INA_CHECK_LAUNCH();
  return 0;
}

}  // namespace ina
