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
